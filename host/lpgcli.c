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
 *   lpgcli --lp MODEL [--big-m] [--rule ...]     the reference's model format,
 *          through the C front end (lpfront.c) onto the device
 *   lpgcli --lp-dump MODEL                       the SimplexMatrix as JSON (no device)
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

#include "lpfront.h"
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

static char *read_all(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        printf("File not readable or does not exist.\n");   /* main.c:41 wording */
        return NULL;
    }
    size_t cap = 4096, n = 0;
    char *b = (char *)malloc(cap);
    for (size_t r; b && (r = fread(b + n, 1, cap - n - 1, f)) > 0;) {
        n += r;
        if (n + 1 == cap) b = (char *)realloc(b, cap *= 2);
    }
    fclose(f);
    if (b) b[n] = '\0';
    return b;
}

/* a JSON string literal: quotes, backslashes and control characters escaped
 * (error messages and variable names carry text from the model file) */
static void json_str(const char *t) {
    putchar('"');
    for (const unsigned char *c = (const unsigned char *)t; *c; c++) {
        if (*c == '"' || *c == '\\') printf("\\%c", *c);
        else if (*c == '\n') printf("\\n");
        else if (*c == '\t') printf("\\t");
        else if (*c < 0x20) printf("\\u%04x", *c);
        else putchar(*c);
    }
    putchar('"');
}

static void print_error(const char *err) {
    printf("{\"error\": ");
    json_str(err);
    printf("}\n");
}

static void print_q(lpf_q q) { printf("\"%lld/%lld\"", (long long)q.num, (long long)q.den); }

/* the reference model file -> SimplexMatrix (dump) or the device optimum */
static int run_lp(const char *path, int dump, int bigm, int rule, int device) {
    char err[512] = "";
    char *text = read_all(path);
    if (!text) return 1;
    lpf_smatrix sm;
    const int rc = lpf_build(text, &sm, err, sizeof err);
    free(text);
    if (rc) {
        print_error(err);
        return 3;
    }
    if (dump) {
        printf("{\"names\": [");
        for (int64_t j = 0; j < sm.n; j++) {
            char nm[256];
            snprintf(nm, sizeof nm, "%s%s", sm.names[j], sm.inverted[j] ? "'" : "");
            printf("%s", j ? ", " : "");
            json_str(nm);
        }
        printf("], \"basis\": [");
        for (int64_t i = 0; i < sm.m; i++) printf("%s%lld", i ? ", " : "", (long long)sm.basis[i]);
        printf("], \"costs\": [");
        for (int64_t j = 0; j < sm.n; j++) {
            if (j) printf(", ");
            print_q(sm.costs[j]);
        }
        printf("], \"constant\": ");
        print_q(sm.constant);
        printf(", \"zcoef\": ");
        print_q(sm.zcoef);
        printf(", \"rows\": [");
        for (int64_t i = 0; i < sm.m; i++) {
            printf("%s[", i ? ", " : "");
            for (int64_t j = 0; j <= sm.n; j++) {
                if (j) printf(", ");
                print_q(sm.rows[i * (sm.n + 1) + j]);
            }
            printf("]");
        }
        printf("], \"vars\": [");
        for (int64_t v = 0; v < sm.nvars; v++) {
            printf("%s[", v ? ", " : "");
            json_str(sm.vars[v].name);
            printf(", %d, ", sm.vars[v].relation);
            json_str(sm.vars[v].former);
            printf(", ");
            json_str(sm.vars[v].latter);
            printf("]");
        }
        printf("]}\n");
        lpf_free(&sm);
        return 0;
    }
    lpf_solution sol;
    if (lpf_solve(&sm, bigm, rule, device, &sol, err, sizeof err)) {
        print_error(err);
        lpf_free(&sm);
        return 1;
    }
    printf("{\"status\": \"%s\", \"pivots\": %lld", status_name(sol.status), (long long)sol.pivots);
    if (sol.status == LPG_OPTIMAL) {
        printf(", \"z\": %.17g, \"variables\": {", sol.z);
        for (int64_t v = 0; v < sm.nvars; v++) {
            printf("%s", v ? ", " : "");
            json_str(sm.vars[v].name);
            printf(": %.17g", sol.vals[v]);
        }
        printf("}");
    }
    printf("}\n");
    lpf_solution_free(&sol);
    lpf_free(&sm);
    return 0;
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
    const char *file = NULL, *lpfile = NULL;
    int dump = 0, bigm = 0;
    for (int a = 1; a < argc; a++) {
        if (!strcmp(argv[a], "--synthetic") && a + 2 < argc) {
            m = atoll(argv[++a]);
            n = atoll(argv[++a]);
        } else if (!strcmp(argv[a], "--tableau") && a + 1 < argc) {
            file = argv[++a];
        } else if ((!strcmp(argv[a], "--lp") || !strcmp(argv[a], "--lp-dump")) && a + 1 < argc) {
            dump = !strcmp(argv[a], "--lp-dump");
            lpfile = argv[++a];
        } else if (!strcmp(argv[a], "--big-m")) {
            bigm = 1;
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
    if (lpfile) return run_lp(lpfile, dump, bigm, rule, device);
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
