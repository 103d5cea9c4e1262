/*
 * lpg_bridge.c — the binding that puts the gfx950 pivot engine behind the
 * reference's own CLI (SomeBottle/LinearProgramming), unmodified.
 *
 * The reference's newSimplex (Source/simplex.c:27-73) builds the tableau with
 * CreateSMatrix (simplex.c:40; Source/matrix.c:19-91) and then frees it
 * without pivoting (simplex.c:65-67). This file supplies the missing step.
 * Here it is linked around the untouched reference sources with
 * `-Wl,--wrap=CreateSMatrix` (integration/Makefile), so every tableau the
 * reference builds is handed to include/lpg.h before the reference continues;
 * a maintainer adopting the engine would instead call LPGSolveSMatrix() from
 * simplex.c:40 directly.
 *
 * Artificials: rows without a unit basic column are given artificial columns
 * and solved by two-phase (default) or Big-M (LPG_ARTIFICIAL=bigm).
 *
 * Conversion (SURVEY.md §8(b) "build-side caller"): every cell through the
 * reference's own Decimalize (Source/basicFuncs.c:298-313), the basis from
 * SimplexMatrix.basicVars (which alias varNames, matrix.c:76-77), costs from
 * ofCosts (matrix.c:55-57). Readout (§8(a) a14): x_B = column 0, z + the
 * objective constant CreateSMatrix strips (matrix.c:23-28), sign flipped back
 * for a min problem (simplex.c:99-106), x = -x' for inverted x <= 0 variables
 * (simplex.c:343-354) and x = x'' - x' for free variables (simplex.c:110-169).
 */
#include <stdint.h>

#include "public.h"
#include "matrix.h"
#include "lpg.h"

SimplexMatrix __real_CreateSMatrix(LPModel *model, size_t **lack, short int *valid);

static double value_of(const char *name, char **varNames, const double *x, size_t ofLen) {
    size_t j;
    for (j = 0; j < ofLen; j++)
        if (strcmp(varNames[j], name) == 0) return x[j];
    return 0.0;
}

/* Solve one CreateSMatrix tableau on the device and print the optimum in the
 * reference's style. Rows without a true unit basic column (CreateSMatrix's
 * lack list, matrix.c:80-89, and rows whose "identity" column fails the unit
 * test, the quirk of matrix.c:67-78) get artificial columns appended and are
 * solved by the two-phase method (default) or Big-M (LPG_ARTIFICIAL=bigm),
 * the two choices the reference's menu offers (simplex.c:45-55).
 * Returns 1 (valid) on success, 0 otherwise. */
short int LPGSolveSMatrix(SimplexMatrix *mx, double constant, double zcoef, short int *inverted) {
    const int64_t m = (int64_t) mx->basicLen, nc0 = (int64_t) mx->ofLen + 1;
    size_t i, j;
    short int valid = 0;
    int64_t *basis = (int64_t *) calloc((size_t) m, sizeof(int64_t));
    int64_t nlack = 0;
    for (i = 0; i < (size_t) m; i++) {
        for (j = 0; j < mx->ofLen; j++)
            if (mx->basicVars[i] == mx->varNames[j]) basis[i] = (int64_t) j + 1;
        if (basis[i]) {   /* keep it only if it is a true unit column */
            size_t q;
            for (q = 0; q < (size_t) m; q++)
                if (Decimalize(*mx->cMatrix[q][basis[i]]) != (q == i ? 1.0 : 0.0)) basis[i] = 0;
        }
        if (!basis[i]) nlack++;
    }
    const int64_t nc = nc0 + nlack;                 /* artificials appended after the original columns */
    double *rows = (double *) calloc((size_t) (m * nc), sizeof(double));
    double *cost = (double *) calloc((size_t) nc, sizeof(double));
    double *xB = (double *) calloc((size_t) m, sizeof(double));
    double *x = (double *) calloc((size_t) nc, sizeof(double));
    lpg_ctx *ctx = NULL;
    int64_t a = nc0;
    for (i = 0; i < (size_t) m; i++) {
        for (j = 0; j < (size_t) nc0; j++)
            rows[i * nc + j] = Decimalize(*mx->cMatrix[i][j]);
        if (!basis[i]) {
            rows[i * nc + a] = 1.0;
            basis[i] = a++;
        }
    }
    for (j = 0; j < mx->ofLen; j++) cost[j] = Decimalize(*mx->ofCosts[j]);
    const char *method = getenv("LPG_ARTIFICIAL");
    const int bigm = nlack > 0 && method && strcmp(method, "bigm") == 0;
    int rc;
    lpg_result res;
    if ((rc = lpg_create(&ctx, 0, m, nc, bigm ? LPG_FLAG_BIG_M : 0)) != 0 ||
        (rc = lpg_load_rows(ctx, 0, m, rows, nc)) != 0 || (rc = lpg_set_basis(ctx, basis)) != 0) {
        printf("ERROR: device simplex failed: %s\n", lpg_last_error(ctx));
        goto out;
    }
    if (nlack == 0)
        rc = lpg_set_objective(ctx, cost) || lpg_solve(ctx, (int64_t) 1 << 40, LPG_RULE_DANTZIG, &res);
    else if (bigm)
        rc = lpg_solve_big_m(ctx, nc0, cost, (int64_t) 1 << 40, LPG_RULE_DANTZIG, &res);
    else
        rc = lpg_solve_two_phase(ctx, nc0, cost, (int64_t) 1 << 40, LPG_RULE_DANTZIG, &res);
    if (rc != 0 || lpg_get_column0(ctx, xB) != 0 || lpg_get_basis(ctx, basis) != 0) {
        printf("ERROR: device simplex failed: %s\n", lpg_last_error(ctx));
        goto out;
    }
    printf("\n---------------\n> Device Simplex (gfx950, lpg)%s\n\n",
           nlack == 0 ? "" : (bigm ? ", Big-M (symbolic M)" : ", two-phase"));
    if (res.status == LPG_UNBOUNDED) {
        printf("The LP is UNBOUNDED (after %lld pivots).\n", (long long) res.pivots);
        valid = 1;
        goto out;
    }
    if (res.status == LPG_INFEASIBLE) {
        printf("The LP is INFEASIBLE (after %lld pivots).\n", (long long) res.pivots);
        valid = 1;
        goto out;
    }
    if (res.status != LPG_OPTIMAL) {
        printf("Stopped with status %d after %lld pivots.\n", res.status, (long long) res.pivots);
        goto out;
    }
    for (i = 0; i < (size_t) m; i++) x[basis[i] - 1] = xB[i];
    printf("OPTIMAL after %lld pivots.\n\tz = %.12g\n\t", (long long) res.pivots,
           (res.objective + constant) / zcoef);
    for (j = 0; j < mx->ofLen; j++)
        printf("%s%s=%.12g | ", mx->varNames[j], inverted[j] ? "'" : "", x[j]);
    printf("\nVariables:\n\t");
    {
        short int ok = 1;
        size_t nv = 0;
        VarItem **items = GetVarItems(&nv, &ok);
        for (i = 0; ok && i < nv; i++) {
            VarItem *v = items[i];
            double val;
            if (v->relation == 0 && strlen(v->formerX) > 0)       /* x = x'' - x' */
                val = value_of(v->formerX, mx->varNames, x, mx->ofLen) -
                      value_of(v->latterX, mx->varNames, x, mx->ofLen);
            else if (v->relation < 0 && v->number == 0)           /* x = -x' */
                val = -value_of(v->keyName, mx->varNames, x, mx->ofLen);
            else
                val = value_of(v->keyName, mx->varNames, x, mx->ofLen);
            printf("%s=%.12g | ", v->keyName, val);
        }
        free(items);
    }
    printf("\n");
    valid = 1;
out:
    lpg_destroy(ctx);
    free(rows);
    free(cost);
    free(xB);
    free(x);
    free(basis);
    return valid;
}

SimplexMatrix __wrap_CreateSMatrix(LPModel *model, size_t **lack, short int *valid) {
    size_t j;
    double constant = 0.0;
    /* CreateSMatrix drops the objective constant (matrix.c:23-28): keep it. */
    for (j = 0; j < model->objective.rightLen; j++)
        if (strlen(model->objective.right[j]->variable) == 0)
            constant += Decimalize(model->objective.right[j]->coefficient);
    const double zcoef = Decimalize(model->objective.left[0]->coefficient);
    SimplexMatrix mx = __real_CreateSMatrix(model, lack, valid);
    {   /* lacking rows are handled with artificials (the reference then still shows its menu) */
        short int *inv = (short int *) calloc(mx.ofLen + 1, sizeof(short int));
        for (j = 0; j < mx.ofLen && j < model->objective.rightLen; j++)
            inv[j] = model->objective.right[j]->inverted;
        LPGSolveSMatrix(&mx, constant, zcoef, inv);
        free(inv);
    }
    return mx;
}
