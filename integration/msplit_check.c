/*
 * msplit_check.c -- test driver for the bridge's handling of the symbolic
 * constant M (lpg_bridge.c split_number). The reference's parser refuses M in
 * user input (dataReader.c:413-417), so this driver runs the reference's own
 * front end (Parser, LPTrans, LPStandardize, LPAlign) on an LP file, builds
 * the tableau with the bridge's LPGCreateSMatrix, then gives one variable's
 * cost (or one constraint cell) an M part the way Fractionize represents
 * "pM/q + s" (numOprts.h:15-37: numerator/denominator with constant M in the
 * numerator, sub = s), and solves through LPGSolveSMatrix.
 *
 * usage: msplit_check FILE compare             (LPGCreateSMatrix vs the reference's
 *                                              CreateSMatrix: cells, names, basis,
 *                                              lack, valid; LPs with <= 1 lacking row)
 *        msplit_check FILE cost VAR P Q S      (cost of VAR = (P/Q) M + S)
 *        msplit_check FILE cell ROW VAR         (cell (ROW, VAR) = 1 M: refused)
 *        msplit_check FILE cost-denominator VAR (cost of VAR = 1/M: refused)
 * Test infrastructure only (tests/test_integration_cli.py).
 */
#include "public.h"
#include "matrix.h"
#include "simplex.h"

SimplexMatrix LPGCreateSMatrix(LPModel *model, size_t **lack, short int *valid);
SimplexMatrix __real_CreateSMatrix(LPModel *model, size_t **lack, short int *valid);

static int same_number(const Number *a, const Number *b) {
    return a->numerator == b->numerator && a->denominator == b->denominator && a->constant == b->constant &&
           a->constLies == b->constLies && a->valid == b->valid;
}

/* 0 when the restatement built exactly the reference's SimplexMatrix */
static int compare(LPModel *model) {
    LPModel m1 = CopyModel(model), m2 = CopyModel(model);
    size_t *l1 = NULL, *l2 = NULL, i, j, bad = 0;
    short int v1 = 1, v2 = 1;
    SimplexMatrix a = __real_CreateSMatrix(&m1, &l1, &v1);
    SimplexMatrix b = LPGCreateSMatrix(&m2, &l2, &v2);
    if (a.ofLen != b.ofLen || a.basicLen != b.basicLen || v1 != v2 || (l1 == NULL) != (l2 == NULL) ||
        m1.objective.rightLen != m2.objective.rightLen) {
        printf("MISMATCH shape/valid/lack\n");
        return 1;
    }
    for (j = 0; j < a.ofLen; j++) {
        bad += strcmp(a.varNames[j], b.varNames[j]) != 0;
        bad += !same_number(a.ofCosts[j], b.ofCosts[j]);
    }
    for (i = 0; i < a.basicLen; i++) {
        for (j = 0; j <= a.ofLen; j++) bad += !same_number(a.cMatrix[i][j], b.cMatrix[i][j]);
        bad += (a.basicVars[i] == NULL) != (b.basicVars[i] == NULL);
        if (a.basicVars[i] && b.basicVars[i]) bad += strcmp(a.basicVars[i], b.basicVars[i]) != 0;
        if (l1 && l2) bad += l1[i] != l2[i];
    }
    printf("compare: %zu rows x %zu columns, valid=%d, lack=%s, mismatches=%zu\n", a.basicLen, a.ofLen, v1,
           l1 ? "yes" : "no", bad);
    RevokeSMatrix(&a);
    RevokeSMatrix(&b);
    free(l1);
    free(l2);
    FreeModel(&m1);
    FreeModel(&m2);
    return bad != 0;
}
short int LPGSolveSMatrix(SimplexMatrix *mx, double constant, double zcoef, short int *inverted);

static size_t column_of(const SimplexMatrix *mx, const char *name) {
    size_t j;
    for (j = 0; j < mx->ofLen; j++)
        if (strcmp(mx->varNames[j], name) == 0) return j;
    fprintf(stderr, "no variable %s\n", name);
    exit(2);
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    FILE *fp = fopen(argv[1], "r");
    if (!fp) return 2;
    InitVarDict();
    LPModel parsed = Parser(fp);
    LPTrans(&parsed);
    if (!parsed.valid) return 3;
    LPModel model = CopyModel(&parsed);
    LPStandardize(&model, 0);
    LPAlign(&model);
    if (strcmp(argv[2], "compare") == 0) return compare(&model);
    size_t j, *lack = NULL;
    short int valid = 1;
    double constant = 0.0;
    for (j = 0; j < model.objective.rightLen; j++)
        if (strlen(model.objective.right[j]->variable) == 0)
            constant += Decimalize(model.objective.right[j]->coefficient);
    const double zcoef = Decimalize(model.objective.left[0]->coefficient);
    SimplexMatrix mx = LPGCreateSMatrix(&model, &lack, &valid);
    Constant *M = &constants[0];   /* the parser's one constant, 'M' (dataReader.c:165-173) */
    if (strcmp(argv[2], "cost") == 0 && argc == 7) {
        Number *c = mx.ofCosts[column_of(&mx, argv[3])];
        c->numerator = atol(argv[4]);
        c->denominator = atol(argv[5]);
        c->constant = M;
        c->constLies = 0;
        c->sub.numerator = atol(argv[6]);
        c->sub.denominator = 1;
        c->sub.valid = 1;
    } else if (strcmp(argv[2], "cell") == 0 && argc == 5) {
        Number *c = mx.cMatrix[atol(argv[3])][column_of(&mx, argv[4]) + 1];
        c->numerator = 1;
        c->denominator = 1;
        c->constant = M;
        c->constLies = 0;
    } else if (strcmp(argv[2], "cost-denominator") == 0 && argc == 4) {
        Number *c = mx.ofCosts[column_of(&mx, argv[3])];
        c->numerator = 1;
        c->denominator = 1;
        c->constant = M;
        c->constLies = 1;
    } else {
        return 2;
    }
    short int *inv = (short int *) calloc(mx.ofLen + 1, sizeof(short int));
    for (j = 0; j < mx.ofLen && j < model.objective.rightLen; j++) inv[j] = model.objective.right[j]->inverted;
    const short int ok = LPGSolveSMatrix(&mx, constant, zcoef, inv);
    printf("\nvalid=%d\n", ok);
    free(inv);
    free(lack);
    RevokeSMatrix(&mx);
    FreeModel(&model);
    FreeModel(&parsed);
    fclose(fp);
    return 0;
}
