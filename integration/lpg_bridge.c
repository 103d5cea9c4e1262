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
 * CreateSMatrix itself is restated here (LPGCreateSMatrix, matrix.c:19-91):
 * the reference's copy writes the lack list through `*lack[lackPtr++]`
 * (matrix.c:86), i.e. through the caller's pointer variable and the stack
 * words after it, so any LP with two or more rows lacking a unit column
 * crashed before the engine was reached. The
 * restatement builds the same SimplexMatrix (cells, names, costs, the
 * identity heuristic of matrix.c:67-78 with its quirk, valid / lack) and
 * fills the lack list correctly.
 *
 * Conversion (SURVEY.md §8(b) "build-side caller"): every cell through the
 * reference's own Decimalize (Source/basicFuncs.c:298-313) -- except a Number
 * carrying the constant M (numOprts.h:15-37: value = (num/den) M + sub),
 * which Decimalize turns into 0 with a printf. A cost with M in its
 * numerator is split into the pair (num/den, sub) and solved on a Big-M
 * context (M part first, lexicographically); M in a denominator or in a
 * constraint cell is refused with an ERROR (valid = 0). (The reference's own
 * parser rejects M in user input, dataReader.c:413-417, so only a caller
 * building the SimplexMatrix itself can get here with M.) The basis from
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

SimplexMatrix LPGCreateSMatrix(LPModel *model, size_t **lack, short int *valid);

/* A Number as (M part, real part): value = (num/den) M + sub when the constant
 * M sits in the numerator (numOprts.h:15-37, Fractionize basicFuncs.c:165-291);
 * plain numbers go through the reference's own Decimalize. Returns 0, or -1
 * for an invalid number or M in a denominator (an infinitesimal M^-1 part,
 * which two objective rows cannot hold). */
static int split_number(Number v, double *mpart, double *rpart) {
    if (!v.valid) return -1;
    if (v.constant == NULL) {
        *mpart = 0.0;
        *rpart = Decimalize(v);
        return 0;
    }
    if (v.constLies != 0 || v.denominator == 0) return -1;
    *mpart = (double) v.numerator / (double) v.denominator;
    *rpart = (v.sub.valid && v.sub.denominator) ? (double) v.sub.numerator / (double) v.sub.denominator : 0.0;
    return 0;
}

static Number *copy_number(Number v) {
    Number *p = (Number *) calloc(1, sizeof(Number));
    *p = v;
    return p;
}

/* Clean-room restatement of CreateSMatrix (matrix.c:19-91) with the lack list
 * written correctly. Inputs and outputs as the reference's:
 *  - the objective's constant term (empty variable name) is removed from the
 *    model (matrix.c:23-28; the bridge reads it before calling this);
 *  - cMatrix[i] = [b_i | a_i1 .. a_iN] as heap Number copies, varNames /
 *    ofCosts per objective term, basicVars / basicCosts aliasing them;
 *  - identity heuristic: column j is basic in row p when the sum over its
 *    entries of (e >= 0 ? (int) e : 6) is 1, p being the last row with e == 1
 *    (row 0 if none), a later column replacing an earlier one in the same
 *    row -- including the accepted (3/2, 1/2) quirk, which the solver below
 *    re-checks;
 *  - rows left without a basic variable: *lack = calloc'd list of their
 *    indices (caller frees), *valid = 0; otherwise *lack = NULL and *valid is
 *    left as the caller set it. */
SimplexMatrix LPGCreateSMatrix(LPModel *model, size_t **lack, short int *valid) {
    SimplexMatrix sm = {0};
    OF *of = &model->objective;
    size_t i, j, nl = 0;
    for (j = of->rightLen; j-- > 0;)
        if (of->right[j]->variable[0] == '\0') of->rightLen = RmvTerm(of->right, of->rightLen, j, 1);
    sm.ofLen = of->rightLen;
    sm.basicLen = model->stLen;
    sm.ofCosts = (Number **) calloc(sm.ofLen, sizeof(Number *));
    sm.varNames = (char **) calloc(sm.ofLen, sizeof(char *));
    sm.cMatrix = (Number ***) calloc(sm.basicLen, sizeof(Number **));
    sm.basicVars = (char **) calloc(sm.basicLen, sizeof(char *));
    sm.basicCosts = (Number **) calloc(sm.basicLen, sizeof(Number *));
    for (i = 0; i < sm.basicLen; i++) {
        sm.cMatrix[i] = (Number **) calloc(sm.ofLen + 1, sizeof(Number *));
        sm.cMatrix[i][0] = copy_number(model->subjectTo[i].right[0]->coefficient);
    }
    for (j = 0; j < sm.ofLen; j++) {
        const Term *t = of->right[j];
        int score = 0;
        size_t row = 0;
        sm.varNames[j] = (char *) calloc(strlen(t->variable) + 1, sizeof(char));
        strcpy(sm.varNames[j], t->variable);
        sm.ofCosts[j] = copy_number(t->coefficient);
        for (i = 0; i < sm.basicLen; i++) {
            Number *cell = copy_number(model->subjectTo[i].left[j]->coefficient);
            const double e = Decimalize(*cell);
            sm.cMatrix[i][j + 1] = cell;
            if (e == 1) row = i;
            score += e >= 0 ? (int) e : 6;
        }
        if (score == 1) {
            sm.basicVars[row] = sm.varNames[j];
            sm.basicCosts[row] = sm.ofCosts[j];
        }
    }
    *lack = NULL;
    for (i = 0; i < sm.basicLen; i++) {
        if (sm.basicVars[i] != NULL) continue;
        if (*lack == NULL) *lack = (size_t *) calloc(sm.basicLen, sizeof(size_t));
        (*lack)[nl++] = i;
        *valid = 0;
    }
    return sm;
}

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
    double zM = 0.0;
    int64_t *basis = (int64_t *) calloc((size_t) m, sizeof(int64_t));
    int64_t nlack = 0;
    for (i = 0; i < (size_t) m; i++) {
        for (j = 0; j < mx->ofLen; j++)
            if (mx->basicVars[i] == mx->varNames[j]) basis[i] = (int64_t) j + 1;
        if (basis[i]) {   /* keep it only if it is a true unit column */
            size_t q;
            for (q = 0; q < (size_t) m; q++)
            {
                double mp = 0.0, rp = 0.0;
                if (split_number(*mx->cMatrix[q][basis[i]], &mp, &rp) != 0 || mp != 0.0 || rp != (q == i ? 1.0 : 0.0))
                    basis[i] = 0;
            }
        }
        if (!basis[i]) nlack++;
    }
    const int64_t nc = nc0 + nlack;                 /* artificials appended after the original columns */
    double *rows = (double *) calloc((size_t) (m * nc), sizeof(double));
    double *cost = (double *) calloc((size_t) nc, sizeof(double));
    double *xB = (double *) calloc((size_t) m, sizeof(double));
    double *x = (double *) calloc((size_t) nc, sizeof(double));
    double *costM = (double *) calloc((size_t) nc, sizeof(double));
    lpg_ctx *ctx = NULL;
    int64_t a = nc0;
    int has_m = 0, rc;
    lpg_result res;
    for (i = 0; i < (size_t) m; i++) {
        for (j = 0; j < (size_t) nc0; j++) {
            double mp = 0.0, rp = 0.0;
            if (split_number(*mx->cMatrix[i][j], &mp, &rp) != 0 || mp != 0.0) {
                printf("ERROR: device simplex: cell (%zu, %zu) is not a plain number (the constant M is only "
                       "supported in objective costs)\n", i, j);
                goto out;
            }
            rows[i * nc + j] = rp;
        }
        if (!basis[i]) {
            rows[i * nc + a] = 1.0;
            basis[i] = a++;
        }
    }
    for (j = 0; j < mx->ofLen; j++)
        if (split_number(*mx->ofCosts[j], &costM[j], &cost[j]) != 0) {
            printf("ERROR: device simplex: cost of %s is invalid or has M in a denominator\n", mx->varNames[j]);
            goto out;
        } else if (costM[j] != 0.0) {
            has_m = 1;
        }
    const char *method = getenv("LPG_ARTIFICIAL");
    const int bigm = has_m || (nlack > 0 && method && strcmp(method, "bigm") == 0);
    if ((rc = lpg_create(&ctx, 0, m, nc, bigm ? LPG_FLAG_BIG_M : 0)) != 0 ||
        (rc = lpg_load_rows(ctx, 0, m, rows, nc)) != 0 || (rc = lpg_set_basis(ctx, basis)) != 0) {
        printf("ERROR: device simplex failed: %s\n", lpg_last_error(ctx));
        goto out;
    }
    if (has_m) {
        /* Big-M with symbolic costs: the user's M parts, and -M (max form) on
         * every artificial, in the M row; the real parts in the real row */
        for (j = (size_t) nc0 - 1; j < (size_t) nc - 1; j++) costM[j] = -1.0;
        rc = lpg_set_objective_m(ctx, costM) || lpg_set_objective(ctx, cost) ||
             lpg_solve(ctx, (int64_t) 1 << 40, LPG_RULE_DANTZIG, &res);
    } else if (nlack == 0)
        rc = lpg_set_objective(ctx, cost) || lpg_solve(ctx, (int64_t) 1 << 40, LPG_RULE_DANTZIG, &res);
    else if (bigm)
        rc = lpg_solve_big_m(ctx, nc0, cost, (int64_t) 1 << 40, LPG_RULE_DANTZIG, &res);
    else
        rc = lpg_solve_two_phase(ctx, nc0, cost, (int64_t) 1 << 40, LPG_RULE_DANTZIG, &res);
    if (rc != 0 || lpg_get_column0(ctx, xB) != 0 || lpg_get_basis(ctx, basis) != 0) {
        printf("ERROR: device simplex failed: %s\n", lpg_last_error(ctx));
        goto out;
    }
    if (has_m && (res.status == LPG_OPTIMAL || res.status == LPG_UNBOUNDED)) {
        /* an artificial left positive: infeasible, at an optimum and at a ray
         * alike, with lpg_solve_big_m's tolerance (relative to sum |x_B|) */
        double bsum = 0.0;
        for (i = 0; i < (size_t) m; i++) bsum += fabs(xB[i]);
        for (i = 0; i < (size_t) m; i++)
            if (basis[i] >= nc0 && xB[i] > 1e-9 * (bsum > 1.0 ? bsum : 1.0)) res.status = LPG_INFEASIBLE;
        if (res.status == LPG_OPTIMAL) {
            if (lpg_get_rows(ctx, m, 1, rows, nc) != 0) goto out;   /* the M row: z = zM M + zR */
            zM = rows[0];
        }
    }
    printf("\n---------------\n> Device Simplex (gfx950, lpg)%s\n\n",
           bigm ? ", Big-M (symbolic M)" : (nlack == 0 ? "" : ", two-phase"));
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
    if (zM != 0.0)
        printf("OPTIMAL after %lld pivots.\n\tz = %.12gM + %.12g\n\t", (long long) res.pivots, zM / zcoef,
               (res.objective + constant) / zcoef);
    else
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
    free(costM);
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
    SimplexMatrix mx = LPGCreateSMatrix(model, lack, valid);   /* not __real_: matrix.c:86 */
    {   /* lacking rows are handled with artificials (the reference then still shows its menu) */
        short int *inv = (short int *) calloc(mx.ofLen + 1, sizeof(short int));
        for (j = 0; j < mx.ofLen && j < model->objective.rightLen; j++)
            inv[j] = model->objective.right[j]->inverted;
        LPGSolveSMatrix(&mx, constant, zcoef, inv);
        free(inv);
    }
    return mx;
}
