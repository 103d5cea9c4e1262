/*
 * lpgcli.c — plain-C host driver of the gfx950 pivot engine (include/lpg.h).
 *
 * The reference's host (Source/main.c:4-45 -> router.c:13-43 ->
 * simplex.c:27-73) is interactive and stops at the tableau. This is the
 * non-interactive driver SURVEY.md §5 (config / flags) asks for, in the
 * reference's own language: it builds or reads a tableau, calls the C-ABI and
 * prints one JSON line, so nothing blocks on stdin.
 *
 *   lpgcli --synthetic M N [--seed S] [--kind dense|degenerate]
 *          [--rule dantzig|bland] [--pivots K] [--device D]
 *   lpgcli --tableau FILE [--rule ...] [--pivots K]
 *
 * FILE: "m ncols" then m+1 rows of ncols numbers ([b | a_1..a_N], objective
 * row last, d_j = z_j - c_j), then m basic columns (1-based).
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lpg.h"

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static const char *status_name(int s) {
    static const char *names[] = {"RUNNING", "OPTIMAL", "UNBOUNDED", "INFEASIBLE", "ITER_LIMIT", "NUMERIC"};
    return (s >= 0 && s <= 5) ? names[s] : "UNKNOWN";
}

static int usage(const char *argv0) {
    fprintf(stderr, "Usage:\n\t%s --synthetic M N [--seed S] [--kind dense|degenerate] [--rule dantzig|bland]"
                    " [--pivots K] [--device D]\n\t%s --tableau FILE [--rule dantzig|bland] [--pivots K]\n",
            argv0, argv0);
    return 2;
}

static int load_tableau_file(lpg_ctx **ctx, const char *path, int device) {
    FILE *f = fopen(path, "r");
    if (!f) {
        printf("File not readable or does not exist.\n");   /* main.c:41 wording */
        return -1;
    }
    long long m = 0, nc = 0;
    if (fscanf(f, "%lld %lld", &m, &nc) != 2 || m < 1 || nc < 2) {
        fclose(f);
        fprintf(stderr, "ERROR: bad tableau header\n");
        return -1;
    }
    double *rows = (double *)malloc((size_t)((m + 1) * nc) * sizeof(double));
    int64_t *basis = (int64_t *)malloc((size_t)m * sizeof(int64_t));
    int ok = rows && basis;
    for (long long q = 0; ok && q < (m + 1) * nc; q++) ok = fscanf(f, "%lf", &rows[q]) == 1;
    for (long long q = 0; ok && q < m; q++) {
        long long b;
        ok = fscanf(f, "%lld", &b) == 1;
        basis[q] = b;
    }
    fclose(f);
    int rc = -1;
    if (!ok) {
        fprintf(stderr, "ERROR: truncated tableau file\n");
    } else if ((rc = lpg_create(ctx, device, m, nc, 0)) != 0 ||
               (rc = lpg_load_rows(*ctx, 0, m + 1, rows, nc)) != 0 ||
               (rc = lpg_set_basis(*ctx, basis)) != 0) {
        fprintf(stderr, "ERROR: %s\n", lpg_last_error(*ctx));
    }
    free(rows);
    free(basis);
    return rc;
}

int main(int argc, char **argv) {
    long long m = 0, n = 0, pivots = (long long)1 << 40;
    unsigned long long seed = 20220518ull;
    int kind = LPG_GEN_DENSE, rule = LPG_RULE_DANTZIG, device = 0;
    const char *file = NULL;
    for (int a = 1; a < argc; a++) {
        if (!strcmp(argv[a], "--synthetic") && a + 2 < argc) {
            m = atoll(argv[++a]);
            n = atoll(argv[++a]);
        } else if (!strcmp(argv[a], "--tableau") && a + 1 < argc) {
            file = argv[++a];
        } else if (!strcmp(argv[a], "--seed") && a + 1 < argc) {
            seed = strtoull(argv[++a], NULL, 10);
        } else if (!strcmp(argv[a], "--kind") && a + 1 < argc) {
            kind = !strcmp(argv[++a], "degenerate") ? LPG_GEN_DEGENERATE : LPG_GEN_DENSE;
        } else if (!strcmp(argv[a], "--rule") && a + 1 < argc) {
            rule = !strcmp(argv[++a], "bland") ? LPG_RULE_BLAND : LPG_RULE_DANTZIG;
        } else if (!strcmp(argv[a], "--pivots") && a + 1 < argc) {
            pivots = atoll(argv[++a]);
        } else if (!strcmp(argv[a], "--device") && a + 1 < argc) {
            device = atoi(argv[++a]);
        } else {
            return usage(argv[0]);
        }
    }
    lpg_ctx *ctx = NULL;
    int rc;
    if (file) {
        if (load_tableau_file(&ctx, file, device) != 0) {
            lpg_destroy(ctx);
            return 1;
        }
    } else if (m > 0 && n > 0) {
        if ((rc = lpg_create(&ctx, device, m, n + m + 1, 0)) != 0 || (rc = lpg_generate(ctx, n, seed, kind)) != 0) {
            fprintf(stderr, "ERROR: %s\n", lpg_last_error(ctx));
            lpg_destroy(ctx);
            return 1;
        }
    } else {
        return usage(argv[0]);
    }
    lpg_result res;
    const double t0 = now();
    rc = lpg_solve(ctx, pivots, rule, &res);
    const double dt = now() - t0;
    if (rc != 0) {
        fprintf(stderr, "ERROR: %s\n", lpg_last_error(ctx));
        lpg_destroy(ctx);
        return 1;
    }
    lpg_info_t info;
    lpg_info(ctx, &info);
    printf("{\"status\": \"%s\", \"pivots\": %lld, \"objective\": %.17g, \"seconds\": %.6f, "
           "\"pivots_per_s\": %.3f, \"m\": %lld, \"ncols\": %lld, \"rule\": \"%s\"}\n",
           status_name(res.status), (long long)res.pivots, res.objective, dt, dt > 0 ? (double)res.pivots / dt : 0.0,
           (long long)info.m, (long long)info.ncols, rule == LPG_RULE_BLAND ? "bland" : "dantzig");
    lpg_destroy(ctx);
    return 0;
}
