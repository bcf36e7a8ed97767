/* TEST INFRASTRUCTURE: AddressSanitizer + UndefinedBehaviorSanitizer driver for the CPU oracle.
 * Built by tests/native/Makefile (target oracle_sanitize) as one translation unit with
 * oracle/lafse3_oracle.c, run by tests/test_sanitizers.py.  Exercises every exported entry point on a
 * small seeded batch (written by the test as raw float64: B, then ini B x 13, goal B x 3, gate12 B x 12,
 * dnn_out B x 7): both gradient modes, a shorter horizon, u_last, the reward/collision scorer, the
 * model and cost derivatives, the trace/dump debug hooks.  Any sanitizer report aborts with a
 * non-zero exit (-fno-sanitize-recover=all); the values are checked by the other tests. */
#include "../../oracle/lafse3_oracle.c"

#include <stdio.h>

static int all_finite(const double *v, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        if (!isfinite(v[i])) return 0;
    return 1;
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s inputs.bin\n", argv[0]);
        return 2;
    }
    FILE *fp = fopen(argv[1], "rb");
    if (!fp) return 2;
    double hdr;
    if (fread(&hdr, sizeof(double), 1, fp) != 1) return 2;
    const int64_t B = (int64_t)hdr;
    double *in = malloc(sizeof(double) * (size_t)B * (13 + 3 + 12 + 7));
    if (fread(in, sizeof(double), (size_t)B * 35, fp) != (size_t)B * 35) return 2;
    fclose(fp);
    const double *ini = in, *goal = in + B * 13, *g12 = in + B * 16, *dn = in + B * 28;
    float *dnn = malloc(sizeof(float) * (size_t)B * 7);
    for (int64_t i = 0; i < B * 7; ++i) dnn[i] = (float)dn[i];

    orc_params P;
    orc_default_params(&P);
    const int N = P.horizon;
    double *out8 = malloc(sizeof(double) * B * 8), *R = malloc(sizeof(double) * B * 9);
    int32_t *st = malloc(sizeof(int32_t) * B * 9);
    double *ul = malloc(sizeof(double) * B * 4);
    for (int64_t i = 0; i < B * 4; ++i) ul[i] = 1.0 + 0.1 * (double)(i % 4);

    /* sol_gradient: FD (with and without u_last) and IFT */
    int bad = 0;
    bad |= orc_sol_gradient(&P, B, ini, goal, g12, dnn, NULL, out8, R, st);
    bad |= !all_finite(out8, B * 8);
    bad |= orc_sol_gradient(&P, B, ini, goal, g12, dnn, ul, out8, NULL, NULL);
    P.grad_mode = 1;
    bad |= orc_sol_gradient(&P, B, ini, goal, g12, dnn, NULL, out8, R, st);
    bad |= !all_finite(out8, B * 8);
    P.grad_mode = 0;

    /* solve_q on the nominal parameters, with the debug trace / dump hooks armed */
    double *p = malloc(sizeof(double) * B * 9 * 3), *q = malloc(sizeof(double) * B * 9 * 4);
    double *t = malloc(sizeof(double) * B * 9);
    int32_t *uu = malloc(sizeof(int32_t) * B * 9);
    bad |= orc_grad_params(&P, B, dnn, p, q, t, uu);
    bad |= orc_assemble(&P, B, R, dnn, out8);
    double *x = malloc(sizeof(double) * B * (N + 1) * NX), *u = malloc(sizeof(double) * B * N * NU);
    double *lam = malloc(sizeof(double) * B * N * NX), *cost = malloc(sizeof(double) * B);
    int32_t *cnt = malloc(sizeof(int32_t) * B * 3);
    double *pn = malloc(sizeof(double) * B * 3), *qn = malloc(sizeof(double) * B * 4), *tn = malloc(sizeof(double) * B);
    for (int64_t b = 0; b < B; ++b) {
        memcpy(pn + 3 * b, p + b * 27, sizeof(double) * 3);
        memcpy(qn + 4 * b, q + b * 36, sizeof(double) * 4);
        tn[b] = t[b * 9];
    }
    double *trace = calloc(8 * 64, sizeof(double)), *dump = calloc(8192, sizeof(double));
    orc_debug_trace(trace, 8);
    orc_debug_dump(dump, 3, 1);
    bad |= orc_solve_q(&P, 1, ini, goal, pn, qn, tn, NULL, x, u, lam, cost, st, cnt);
    orc_debug_trace(NULL, 0);
    orc_debug_dump(NULL, -1, 0);
    bad |= orc_solve_q(&P, B, ini, goal, pn, qn, tn, ul, x, u, lam, cost, st, cnt);
    bad |= !all_finite(x, B * (N + 1) * NX) || !all_finite(cost, B);

    /* scorer on the solved trajectories */
    int32_t *br = malloc(sizeof(int32_t) * B * 8);
    bad |= orc_reward(&P, B, x, goal, g12, R, br);
    double *tracks = malloc(sizeof(double) * B * (N + 1) * 12), *col = malloc(sizeof(double) * B);
    int32_t *co = malloc(sizeof(int32_t) * B);
    for (int64_t i = 0; i < B * (N + 1) * 12; ++i) tracks[i] = x[i % (B * (N + 1) * NX)];
    bad |= orc_collis_det(B, N, g12, tracks, col, br, co);

    /* model / cost derivatives at the solved points */
    const int64_t n = B * N;
    double *f = malloc(sizeof(double) * n * NX), *A = malloc(sizeof(double) * n * NX * NX);
    double *Bm = malloc(sizeof(double) * n * NX * NU), *Hxx = malloc(sizeof(double) * n * NX * NX);
    double *Hxu = malloc(sizeof(double) * n * NX * NU);
    double *xs = malloc(sizeof(double) * n * NX);
    for (int64_t b = 0; b < B; ++b) memcpy(xs + b * N * NX, x + b * (N + 1) * NX, sizeof(double) * N * NX);
    bad |= orc_model_eval(&P, n, xs, u, lam, f, A, Bm, Hxx, Hxu);
    double *gl = malloc(sizeof(double) * n * 3), *pt = malloc(sizeof(double) * n * 3), *qt = malloc(sizeof(double) * n * 4);
    double *wk = malloc(sizeof(double) * n), *path = malloc(sizeof(double) * n), *tra = malloc(sizeof(double) * n);
    double *grad = malloc(sizeof(double) * n * NX), *hess = malloc(sizeof(double) * n * NX * NX);
    for (int64_t i = 0; i < n; ++i) {
        memcpy(gl + 3 * i, goal + 3 * (i / N), sizeof(double) * 3);
        memcpy(pt + 3 * i, pn + 3 * (i / N), sizeof(double) * 3);
        memcpy(qt + 4 * i, qn + 4 * (i / N), sizeof(double) * 4);
        wk[i] = (double)(i % N);
    }
    bad |= orc_cost_eval(&P, n, xs, gl, pt, qt, wk, path, tra, grad, hess);
    bad |= !all_finite(A, n * NX * NX) || !all_finite(hess, n * NX * NX);

    /* shorter horizon */
    orc_params P20 = P;
    P20.horizon = 20;
    bad |= orc_solve_q(&P20, B, ini, goal, pn, qn, tn, NULL, x, u, lam, cost, st, cnt);

    free(in); free(dnn); free(out8); free(R); free(st); free(ul); free(p); free(q); free(t); free(uu);
    free(x); free(u); free(lam); free(cost); free(cnt); free(pn); free(qn); free(tn); free(trace); free(dump);
    free(br); free(tracks); free(col); free(co); free(f); free(A); free(Bm); free(Hxx); free(Hxu); free(xs);
    free(gl); free(pt); free(qt); free(wk); free(path); free(tra); free(grad); free(hess);
    printf("oracle_sanitize %s (B=%lld)\n", bad ? "FAILED" : "ok", (long long)B);
    return bad ? 1 : 0;
}
