// mfma_f64_probe.hip — does v_mfma_f64_16x16x4_f64 round like the sequential
// fma chain x = fma(a_k, b_k, x), k = 0..3 (the flush's bitwise contract)?
// Layout (cdna_hip_programming.md): A[l&15][k=l>>4], B[k=l>>4][l&15],
// D col = l&15, row = (l>>4) + 4*reg. Tools only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef double d4 __attribute__((ext_vector_type(4)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// per trial t: A 16x4, B 4x16, C 16x16 (row-major) -> D (mfma), R (chain 0..3), Q (chain 3..0)
__global__ void k_probe(const double *A, const double *B, const double *C, double *D, double *R, double *Q) {
    const int t = blockIdx.x, l = threadIdx.x;
    const double *a = A + t * 64, *b = B + t * 64, *c = C + t * 256;
    double av = a[(l & 15) * 4 + (l >> 4)];
    double bv = b[(l >> 4) * 16 + (l & 15)];
    d4 acc;
    for (int r = 0; r < 4; r++) acc[r] = c[((l >> 4) + 4 * r) * 16 + (l & 15)];
    d4 out = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[t * 256 + ((l >> 4) + 4 * r) * 16 + (l & 15)] = out[r];
    for (int e = l; e < 256; e += 64) {
        const int i = e / 16, j = e % 16;
        double x = c[e], y = c[e];
        for (int k = 0; k < 4; k++) x = fma(a[i * 4 + k], b[k * 16 + j], x);
        for (int k = 3; k >= 0; k--) y = fma(a[i * 4 + k], b[k * 16 + j], y);
        R[t * 256 + e] = x;
        Q[t * 256 + e] = y;
    }
}

static uint64_t s = 88172645463325252ull;
static double rnd() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (double)(s >> 11) * 0x1.0p-53; }

int main() {
    const int NT = 4096;
    const size_t nA = NT * 64, nC = NT * 256;
    double *hA = (double *)malloc(nA * 8), *hB = (double *)malloc(nA * 8), *hC = (double *)malloc(nC * 8);
    const char *names[] = {"small integers, exact", "random, C ~ 1", "random, C ~ 1e-12",
                           "subnormal products / C", "signed zeros, exact cancellation", "inf / nan / huge"};
    for (int mode = 0; mode < 6; mode++) {
        for (size_t i = 0; i < nA; i++) {
            if (mode == 0) {
                hA[i] = (double)((int)(rnd() * 16) - 8);
                hB[i] = (double)((int)(rnd() * 16) - 8);
            } else if (mode == 3) {
                hA[i] = (rnd() - 0.5) * 1e-160;
                hB[i] = (rnd() - 0.5) * 1e-150;
            } else if (mode == 4) {
                const double v[] = {0.0, -0.0, 1.0, -1.0, 0.5};
                hA[i] = v[(int)(rnd() * 5)];
                hB[i] = v[(int)(rnd() * 5)];
            } else if (mode == 5) {
                const double v[] = {1e308, -1e308, INFINITY, -INFINITY, NAN, 2.0, 0.0};
                hA[i] = v[(int)(rnd() * 7)];
                hB[i] = rnd() < 0.9 ? (rnd() - 0.5) : v[(int)(rnd() * 7)];
            } else {
                hA[i] = (rnd() - 0.5) * pow(2.0, (int)(rnd() * 40) - 20);
                hB[i] = (rnd() - 0.5) * pow(2.0, (int)(rnd() * 40) - 20);
            }
        }
        for (size_t i = 0; i < nC; i++) {
            if (mode == 0) hC[i] = (double)((int)(rnd() * 64) - 32);
            else if (mode == 1) hC[i] = rnd() - 0.5;
            else if (mode == 2) hC[i] = (rnd() - 0.5) * 1e-12;
            else if (mode == 3) hC[i] = (rnd() - 0.5) * 1e-308;
            else if (mode == 4) { const double v[] = {0.0, -0.0, 1.0, -1.0}; hC[i] = v[(int)(rnd() * 4)]; }
            else hC[i] = rnd() < 0.9 ? rnd() - 0.5 : 1e308;
        }
        double *A, *B, *C, *D, *R, *Q;
        CHK(hipMalloc(&A, nA * 8)); CHK(hipMalloc(&B, nA * 8)); CHK(hipMalloc(&C, nC * 8));
        CHK(hipMalloc(&D, nC * 8)); CHK(hipMalloc(&R, nC * 8)); CHK(hipMalloc(&Q, nC * 8));
        CHK(hipMemcpy(A, hA, nA * 8, hipMemcpyHostToDevice));
        CHK(hipMemcpy(B, hB, nA * 8, hipMemcpyHostToDevice));
        CHK(hipMemcpy(C, hC, nC * 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_probe, dim3(NT), dim3(64), 0, 0, A, B, C, D, R, Q);
        CHK(hipDeviceSynchronize());
        double *hD = (double *)malloc(nC * 8), *hR = (double *)malloc(nC * 8), *hQ = (double *)malloc(nC * 8);
        CHK(hipMemcpy(hD, D, nC * 8, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(hR, R, nC * 8, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(hQ, Q, nC * 8, hipMemcpyDeviceToHost));
        size_t eqR = 0, eqQ = 0, close = 0;
        for (size_t i = 0; i < nC; i++) {
            // bitwise, except that any NaN equals any NaN (payloads are not part of the contract)
            eqR += memcmp(&hD[i], &hR[i], 8) == 0 || (isnan(hD[i]) && isnan(hR[i]));
            eqQ += memcmp(&hD[i], &hQ[i], 8) == 0;
            close += fabs(hD[i] - hR[i]) <= 1e-12 * fmax(1.0, fabs(hR[i]));
        }
        printf("mode %d (%s): %zu elements; mfma == chain k=0..3: %zu; == chain k=3..0: %zu; close (layout ok): %zu\n",
               mode, names[mode], nC, eqR, eqQ, close);
        free(hD); free(hR); free(hQ);
        hipFree(A); hipFree(B); hipFree(C); hipFree(D); hipFree(R); hipFree(Q);
    }
    return 0;
}
