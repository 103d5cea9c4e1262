/*
 * lpgcli.c — plain-C host driver of the gfx950 pivot engine (include/lpg.h).
 *
 * The reference's host (Source/main.c:4-45 -> router.c:13-43 ->
 * simplex.c:27-73) is interactive and stops at the tableau. This is the
 * non-interactive driver SURVEY.md §5 (config / flags) asks for, in the
 * reference's own language: it builds or reads a tableau, calls the C-ABI and
 * prints one JSON line, so nothing blocks on stdin.
 *
 *   lpgcli --synthetic M N [--seed S] [--kind dense|degenerate|artificial]
 *          [--rule dantzig|bland] [--pivots K] [--device D]
 *   lpgcli --tableau FILE [--rule ...] [--pivots K]
 *   lpgcli --lp MODEL [--big-m] [--rule ...]     the reference's model format,
 *          through the C front end (lpfront.c) onto the device
 *   lpgcli --lp-dump MODEL                       the SimplexMatrix as JSON (no device)
 *   --dual  the dual simplex (router option 2, router.c:32-34, which the
 *          reference leaves empty): with --lp, LPStandardize's dual form
 *          (simplex.c:178-179) solved from its slack basis; with --synthetic,
 *          the dual-feasible LPG_GEN_DUAL tableau; with --tableau, the file's
 *          (dual-feasible) basis; also over --gpus P (round 3).
 *   --kind artificial  BASELINE config 5's family (equality rows with
 *          artificial unit columns) solved by the two-phase method
 *          (lpg_solve_two_phase), on one rank or over --gpus P (round 3).
 *   lpgcli --synthetic M N --gpus P [--exchange push|host]
 *          the row partition over P ranks, one process each (forked before
 *          any HIP call; the parent only relays the host-staged collectives
 *          over socketpairs and never touches a GPU); rank r on device
 *          (D + r) mod #devices; rank 0 prints the JSON line
 *
 * FILE: "m ncols" then m+1 rows of ncols numbers ([b | a_1..a_N], objective
 * row last, d_j = z_j - c_j), then m basic columns (1-based).
 */
#define _POSIX_C_SOURCE 200809L
#include <errno.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

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
    fprintf(stderr, "Usage:\n\t%s --synthetic M N [--seed S] [--kind dense|degenerate|artificial] [--rule dantzig|bland]"
                    " [--pivots K] [--device D] [--gpus P [--exchange push|host]]\n"
                    "\t%s --tableau FILE [--rule dantzig|bland] [--pivots K]\n"
                    "\t%s --lp MODEL [--big-m | --dual] [--rule dantzig|bland]\n\t%s --lp-dump MODEL [--dual]\n"
                    "\t(--dual: the dual simplex; also with --synthetic (any --gpus) and --tableau;\n"
                    "\t --kind artificial: the two-phase method)\n",
            argv0, argv0, argv0, argv0);
    return 2;
}

/* FNV-1a over the pivot log (k, r pairs): one number to compare runs by */
static uint64_t log_fnv(lpg_ctx *ctx, int64_t npiv) {
    uint64_t h = 1469598103934665603ull;
    if (npiv <= 0) return h;
    int64_t *k = (int64_t *)malloc((size_t)npiv * sizeof(int64_t)), *r = (int64_t *)malloc((size_t)npiv * sizeof(int64_t));
    const int64_t n = (k && r) ? lpg_get_log(ctx, k, r, npiv) : 0;
    for (int64_t q = 0; q < n && q < npiv; q++) {
        const int64_t v[2] = {k[q], r[q]};
        const unsigned char *b = (const unsigned char *)v;
        for (size_t i = 0; i < sizeof v; i++) h = (h ^ b[i]) * 1099511628211ull;
    }
    free(k);
    free(r);
    return h;
}

/* ---- --gpus P: the row partition from plain C ----------------------------
 * The reference host is one process (Source/main.c:4-45); the north star's
 * row partition wants one process per GPU. The parent forks P ranks before
 * any HIP call (no process ever forks or execs after GPU initialisation) and
 * then only relays the collectives the engine's setup and bootstraps need
 * (lpg_host_comm_ops: allgather, allreduce of doubles) over one socketpair
 * per rank; per pivot the ranks talk through the owner-push exchange
 * (IPC-mapped device buffers, --exchange push, the default) or through these
 * host collectives (--exchange host). Rank r uses device (D + r) mod
 * #devices, so P ranks may share one GPU. */
typedef struct {
    int fd, world, rank;
} hub_link;

static int write_all(int fd, const void *p, size_t n) {
    const char *c = (const char *)p;
    while (n > 0) {
        const ssize_t w = write(fd, c, n);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return -1;
        c += w;
        n -= (size_t)w;
    }
    return 0;
}

static int read_fd(int fd, void *p, size_t n) {
    char *c = (char *)p;
    while (n > 0) {
        const ssize_t r = read(fd, c, n);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return -1;
        c += r;
        n -= (size_t)r;
    }
    return 0;
}

/* one collective: op ('G' allgather, 'R' allreduce f64) and the payload up, the result down */
static int hub_call(hub_link *h, char op, const void *send, size_t bytes, void *recv, size_t rbytes) {
    const uint64_t n = bytes;
    if (write_all(h->fd, &op, 1) || write_all(h->fd, &n, sizeof n) || write_all(h->fd, send, bytes)) return -1;
    return read_fd(h->fd, recv, rbytes);
}

static int cb_allgather(void *user, const void *send, void *recv, size_t bytes) {
    hub_link *h = (hub_link *)user;
    return hub_call(h, 'G', send, bytes, recv, bytes * (size_t)h->world);
}

static int cb_allreduce(void *user, double *buf, size_t count) {
    return hub_call((hub_link *)user, 'R', buf, count * sizeof(double), buf, count * sizeof(double));
}

/* the parent: serve collectives until every rank has hung up; sums in rank order */
static int hub_serve(int world, const int *fds) {
    char **in = (char **)calloc((size_t)world, sizeof(char *));
    int rc = 0;
    for (;;) {
        char op0 = 0;
        uint64_t n0 = 0;
        int eof = 0;
        for (int r = 0; r < world; r++) {
            char op = 0;
            uint64_t n = 0;
            if (read_fd(fds[r], &op, 1) || read_fd(fds[r], &n, sizeof n)) {
                eof++;
                continue;
            }
            if (r == 0 || eof) {
                op0 = op;
                n0 = n;
            }
            if (op != op0 || n != n0 || (op != 'G' && op != 'R') || (op == 'R' && n % 8)) {
                fprintf(stderr, "ERROR: lpgcli --gpus: ranks disagree on a collective\n");
                rc = 1;
                goto done;
            }
            free(in[r]);
            in[r] = (char *)malloc(n ? n : 1);
            if (!in[r] || read_fd(fds[r], in[r], n)) {
                rc = 1;
                goto done;
            }
        }
        if (eof == world) break;                /* every rank finished */
        if (eof) {                              /* a rank left inside a collective: end them all */
            fprintf(stderr, "ERROR: lpgcli --gpus: a rank exited during a collective\n");
            rc = 1;
            goto done;
        }
        if (op0 == 'G') {
            for (int r = 0; r < world; r++)
                for (int q = 0; q < world; q++)
                    if (write_all(fds[r], in[q], n0)) { rc = 1; goto done; }
        } else {
            double *acc = (double *)in[0];
            for (int q = 1; q < world; q++)
                for (uint64_t i = 0; i < n0 / 8; i++) acc[i] += ((double *)in[q])[i];
            for (int r = 0; r < world; r++)
                if (write_all(fds[r], acc, n0)) { rc = 1; goto done; }
        }
    }
done:
    for (int r = 0; r < world; r++) {
        free(in[r]);
        close(fds[r]);
    }
    free(in);
    return rc;
}

typedef struct {
    long long m, n, pivots;
    unsigned long long seed;
    int kind, rule, device, world, push, dual;
} dist_args;

/* the solve a synthetic tableau asks for: the dual on LPG_GEN_DUAL, the
 * two-phase method on LPG_GEN_ARTIFICIAL (its artificial columns start at
 * 1 + n + ceil(m / 2), as lpg_generate lays them out), else the primal */
static int solve_synthetic(lpg_ctx *ctx, long long m, long long n, int kind, int dual, long long pivots, int rule,
                           lpg_result *res) {
    if (dual) return lpg_solve_dual(ctx, pivots, res);
    if (kind == LPG_GEN_ARTIFICIAL) return lpg_solve_two_phase(ctx, 1 + n + (m + 1) / 2, NULL, pivots, rule, res);
    return lpg_solve(ctx, pivots, rule, res);
}

static const char *method_name(int kind, int dual) {
    return dual ? "dual" : kind == LPG_GEN_ARTIFICIAL ? "two-phase" : "primal";
}

static int run_rank(const dist_args *a, int rank, int fd) {
    hub_link h = {fd, a->world, rank};
    int count = 0, rc;
    lpg_ctx *ctx = NULL;
    if (lpg_device_count(&count) != 0 || count < 1) {
        fprintf(stderr, "ERROR: rank %d: no GPU\n", rank);
        return 1;
    }
    const int dev = (a->device + rank) % count;
    lpg_host_comm_ops ops = {&h, cb_allgather, cb_allreduce};
    if ((rc = lpg_create_dist(&ctx, dev, a->world, rank, a->m, a->n + a->m + 1, 0)) != 0 ||
        (rc = lpg_comm_init_host(ctx, &ops)) != 0)
        goto fail;
    if (a->push) {
        /* every rank attaches the owner push, or none does: the attach is
         * refused where ranks share a GPU (lpg.h), possibly on some ranks only
         * (3 ranks on 2 GPUs), so the ranks agree on an ok flag and, if any was
         * refused, all of them rebuild their context on the host collectives
         * (the caller keeps the collectives, lpg.h) -- exchange 0 in the line */
        char mine[LPG_PUSH_HANDLE_BYTES], ok, oks[256];
        char *all = (char *)malloc((size_t)a->world * LPG_PUSH_HANDLE_BYTES);
        if (!all || a->world > 256) { free(all); rc = LPG_ERR_OOM; goto fail; }
        rc = lpg_comm_push_handle(ctx, mine, sizeof mine);
        ok = rc == 0;
        if (cb_allgather(&h, &ok, oks, 1)) { free(all); rc = LPG_ERR_COMM; goto fail; }
        for (int q = 0; q < a->world; q++) ok = ok && oks[q];
        if (ok && cb_allgather(&h, mine, all, sizeof mine)) { free(all); rc = LPG_ERR_COMM; goto fail; }
        if (ok) {
            rc = lpg_comm_init_push(ctx, all, (size_t)a->world * LPG_PUSH_HANDLE_BYTES);
            if (rc) fprintf(stderr, "lpgcli: rank %d: %s; using the host collectives\n", rank, lpg_last_error(ctx));
            ok = rc == 0;
            if (cb_allgather(&h, &ok, oks, 1)) { free(all); rc = LPG_ERR_COMM; goto fail; }
            for (int q = 0; q < a->world; q++) ok = ok && oks[q];
        }
        free(all);
        if (!ok) {
            lpg_destroy(ctx);
            ctx = NULL;
            if ((rc = lpg_create_dist(&ctx, dev, a->world, rank, a->m, a->n + a->m + 1, 0)) != 0 ||
                (rc = lpg_comm_init_host(ctx, &ops)) != 0)
                goto fail;
        }
    }
    if ((rc = lpg_generate(ctx, a->n, a->seed, a->dual ? LPG_GEN_DUAL : a->kind)) != 0) goto fail;
    char one = 1, got[256];
    if (a->world > 256 || cb_allgather(&h, &one, got, 1)) goto fail;   /* start together */
    const double t0 = now();
    lpg_result res;
    if ((rc = solve_synthetic(ctx, a->m, a->n, a->kind, a->dual, a->pivots, a->rule, &res)) != 0) goto fail;
    if (cb_allgather(&h, &one, got, 1)) goto fail;                     /* the slowest rank's end */
    const double dt = now() - t0;
    lpg_info_t info;
    lpg_info(ctx, &info);
    const uint64_t fnv = log_fnv(ctx, res.pivots);
    if (rank == 0)
        printf("{\"status\": \"%s\", \"pivots\": %lld, \"objective\": %.17g, \"seconds\": %.6f, "
               "\"pivots_per_s\": %.3f, \"m\": %lld, \"ncols\": %lld, \"rule\": \"%s\", \"gpus\": %d, "
               "\"exchange\": %d, \"pivot_wg\": %d, \"residency_fallbacks\": %d, \"defer_k\": %d, "
               "\"method\": \"%s\", \"log_fnv\": \"%016llx\"}\n",
               status_name(res.status), (long long)res.pivots, res.objective, dt, dt > 0 ? (double)res.pivots / dt : 0.0,
               (long long)info.m, (long long)info.ncols, a->rule == LPG_RULE_BLAND && !a->dual ? "bland" : "dantzig",
               a->world, info.exchange, info.pivot_wg, info.residency_fallbacks, info.defer_k,
               method_name(a->kind, a->dual), (unsigned long long)fnv);
    fflush(stdout);
    lpg_destroy(ctx);
    close(fd);
    return 0;
fail:
    fprintf(stderr, "ERROR: rank %d: %s\n", rank, lpg_last_error(ctx));
    lpg_destroy(ctx);
    close(fd);
    return 1;
}

static int run_dist(const dist_args *a) {
    int *fds = (int *)calloc((size_t)a->world, sizeof(int));
    pid_t *pid = (pid_t *)calloc((size_t)a->world, sizeof(pid_t));
    if (!fds || !pid) return 1;
    fflush(stdout);
    for (int r = 0; r < a->world; r++) {
        int sv[2];
        if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 1;
        pid[r] = fork();
        if (pid[r] < 0) return 1;
        if (pid[r] == 0) {                      /* rank r: no HIP call happened in this process yet */
            close(sv[0]);
            for (int q = 0; q < r; q++) close(fds[q]);
            _exit(run_rank(a, r, sv[1]));
        }
        close(sv[1]);
        fds[r] = sv[0];
    }
    int rc = hub_serve(a->world, fds);
    for (int r = 0; r < a->world; r++) {
        int st = 0;
        if (rc) kill(pid[r], SIGTERM);
        if (waitpid(pid[r], &st, 0) < 0 || !WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
    }
    free(fds);
    free(pid);
    return rc;
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
static int run_lp(const char *path, int dump, int method, int rule, int device) {
    char err[512] = "";
    char *text = read_all(path);
    if (!text) return 1;
    lpf_smatrix sm;
    const int rc = lpf_build_form(text, method == LPF_DUAL, &sm, err, sizeof err);
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
    if (lpf_solve(&sm, method, rule, device, &sol, err, sizeof err)) {
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
    int kind = LPG_GEN_DENSE, rule = LPG_RULE_DANTZIG, device = 0, gpus = 1, push = 1;
    const char *file = NULL, *lpfile = NULL;
    int dump = 0, bigm = 0, dual = 0;
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
        } else if (!strcmp(argv[a], "--dual")) {
            dual = 1;
        } else if (!strcmp(argv[a], "--seed") && a + 1 < argc) {
            seed = strtoull(argv[++a], NULL, 10);
        } else if (!strcmp(argv[a], "--kind") && a + 1 < argc) {
            ++a;
            kind = !strcmp(argv[a], "degenerate") ? LPG_GEN_DEGENERATE
                   : !strcmp(argv[a], "artificial") ? LPG_GEN_ARTIFICIAL : LPG_GEN_DENSE;
        } else if (!strcmp(argv[a], "--rule") && a + 1 < argc) {
            rule = !strcmp(argv[++a], "bland") ? LPG_RULE_BLAND : LPG_RULE_DANTZIG;
        } else if (!strcmp(argv[a], "--pivots") && a + 1 < argc) {
            pivots = atoll(argv[++a]);
        } else if (!strcmp(argv[a], "--device") && a + 1 < argc) {
            device = atoi(argv[++a]);
        } else if (!strcmp(argv[a], "--gpus") && a + 1 < argc) {
            gpus = atoi(argv[++a]);
        } else if (!strcmp(argv[a], "--exchange") && a + 1 < argc) {
            push = strcmp(argv[++a], "host") != 0;
        } else {
            return usage(argv[0]);
        }
    }
    if (dual && (bigm || kind == LPG_GEN_ARTIFICIAL)) return usage(argv[0]);
    if (lpfile) return run_lp(lpfile, dump, dual ? LPF_DUAL : bigm ? LPF_BIG_M : LPF_TWO_PHASE, rule, device);
    if (gpus > 1) {
        if (!(m > 0 && n > 0) || gpus > m || gpus > 64) return usage(argv[0]);
        const dist_args da = {m, n, pivots, seed, kind, rule, device, gpus, push, dual};
        return run_dist(&da);
    }
    lpg_ctx *ctx = NULL;
    int rc;
    if (file) {
        if (load_tableau_file(&ctx, file, device) != 0) {
            lpg_destroy(ctx);
            return 1;
        }
    } else if (m > 0 && n > 0) {
        if ((rc = lpg_create(&ctx, device, m, n + m + 1, 0)) != 0 ||
            (rc = lpg_generate(ctx, n, seed, dual ? LPG_GEN_DUAL : kind)) != 0) {
            fprintf(stderr, "ERROR: %s\n", lpg_last_error(ctx));
            lpg_destroy(ctx);
            return 1;
        }
    } else {
        return usage(argv[0]);
    }
    lpg_result res;
    const double t0 = now();
    rc = file ? (dual ? lpg_solve_dual(ctx, pivots, &res) : lpg_solve(ctx, pivots, rule, &res))
              : solve_synthetic(ctx, m, n, kind, dual, pivots, rule, &res);
    const double dt = now() - t0;
    if (rc != 0) {
        fprintf(stderr, "ERROR: %s\n", lpg_last_error(ctx));
        lpg_destroy(ctx);
        return 1;
    }
    lpg_info_t info;
    lpg_info(ctx, &info);
    printf("{\"status\": \"%s\", \"pivots\": %lld, \"objective\": %.17g, \"seconds\": %.6f, "
           "\"pivots_per_s\": %.3f, \"m\": %lld, \"ncols\": %lld, \"rule\": \"%s\", \"gpus\": 1, "
           "\"defer_k\": %d, \"method\": \"%s\", \"log_fnv\": \"%016llx\"}\n",
           status_name(res.status), (long long)res.pivots, res.objective, dt, dt > 0 ? (double)res.pivots / dt : 0.0,
           (long long)info.m, (long long)info.ncols, rule == LPG_RULE_BLAND && !dual ? "bland" : "dantzig", info.defer_k,
           file ? (dual ? "dual" : "primal") : method_name(kind, dual), (unsigned long long)log_fnv(ctx, res.pivots));
    lpg_destroy(ctx);
    return 0;
}
