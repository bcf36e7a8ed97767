// Host build of the device model closed forms (csrc/model.hpp) for CPU unit tests.
// Compiled by tests/test_model_host.py with hipcc (host code only; no GPU needed).
#include "model.hpp"

using namespace lafse3;

static lafse3_params defaults()
{
    lafse3_params p{};
    p.mass = 0.5; p.Jx = 0.0023; p.Jy = 0.0023; p.Jz = 0.004; p.arm_l = 0.35; p.c_tau = 0.0245; p.grav = 9.78;
    p.dt = 0.1; p.wrt = 5; p.wqt = 80; p.wthrust = 0.1; p.wrf = 5; p.wvf = 5; p.wqf = 0; p.wwf = 3;
    p.du_weight = 1;
    return p;
}

extern "C" {

// For n points: f (13), A (13x13) and B (13x4) assembled column-by-column from A_times / B_times,
// A^T (13x13) from At_times, B^T from Bt_times, lambda-Hessian (13x13 via Hxx_times on unit vectors
// with zero cost weights) and the q-u coupling vector.
int model_host_eval(int n, const double *x, const double *u, const double *lam, double *f, double *A, double *B,
                    double *At, double *Bt, double *Hl, double *qu)
{
    lafse3_params p = defaults();
    Model M = make_model(p);
    Attitude at{};
    at.trRt = at.trRg = 3.0;
    for (int i = 0; i < n; ++i) {
        const double *xi = x + i * NX, *ui = u + i * NU, *li = lam + i * NX;
        f_cont(M, xi, ui, f + i * NX);
        for (int j = 0; j < NX; ++j) {
            double e[NX] = {0}, o[NX];
            e[j] = 1.0;
            A_times(M, xi, ui, e, o);
            for (int r = 0; r < NX; ++r) A[i * NX * NX + r * NX + j] = o[r];
            At_times(M, xi, ui, e, o);
            for (int r = 0; r < NX; ++r) At[i * NX * NX + r * NX + j] = o[r];
        }
        for (int j = 0; j < NU; ++j) {
            double e[NU] = {0}, o[NX];
            e[j] = 1.0;
            B_times(M, xi, e, o);
            for (int r = 0; r < NX; ++r) B[i * NX * NU + r * NU + j] = o[r];
        }
        for (int j = 0; j < NX; ++j) {
            double e[NX] = {0}, o[NU];
            e[j] = 1.0;
            Bt_times(M, xi, e, o);
            for (int r = 0; r < NU; ++r) Bt[i * NU * NX + r * NX + j] = o[r];
        }
        // lambda part of the Hessian: zero cost weights so only sum lam_i Hess f_d,i remains
        Model M0 = M;
        M0.wrf = M0.wvf = M0.wwf = M0.wrt = M0.wqt = M0.wqf = 0.0;
        StageHess H;
        stage_hessian(M0, at, 1.0, 0.0, xi, ui, li, H);
        for (int j = 0; j < NX; ++j) {
            double e[NX] = {0}, o[NX];
            e[j] = 1.0;
            Hxx_times(H, e, o);
            for (int r = 0; r < NX; ++r) Hl[i * NX * NX + r * NX + j] = o[r];
        }
        for (int r = 0; r < 4; ++r) qu[i * 4 + r] = H.qu[r];
    }
    return 0;
}

// state cost gradient / Hessian (through stage_hessian + Hxx_times with lam = 0)
int model_host_cost(int n, const double *x, const double *goal, const double *ptra, const double *qtra,
                    const double *wk, double *path, double *tra, double *grad, double *hess)
{
    lafse3_params p = defaults();
    Model M = make_model(p);
    for (int i = 0; i < n; ++i) {
        double Rt[9], Rg[9], St[16], Sg[16];
        dcm(qtra + i * 4, Rt);
        attitude_form(Rt, St);
        const double qg[4] = {1, 0, 0, 0};
        dcm(qg, Rg);
        attitude_form(Rg, Sg);
        Attitude at{};
        for (int e = 0; e < 16; ++e) {
            at.St[e] = St[e];
            at.Sg[e] = Sg[e];
        }
        at.trRt = Rt[0] + Rt[4] + Rt[8];
        at.trRg = Rg[0] + Rg[4] + Rg[8];
        const double *xi = x + i * NX;
        path[i] = state_cost(M, at, goal + i * 3, ptra + i * 3, 0.0, xi);
        double full = state_cost(M, at, goal + i * 3, ptra + i * 3, 1.0, xi);
        tra[i] = full - path[i];
        state_cost_grad(M, at, goal + i * 3, ptra + i * 3, wk[i], xi, grad + i * NX);
        double lam0[NX] = {0}, u0[NU] = {0};
        StageHess H;
        stage_hessian(M, at, 1.0, wk[i], xi, u0, lam0, H);
        for (int j = 0; j < NX; ++j) {
            double e[NX] = {0}, o[NX];
            e[j] = 1.0;
            Hxx_times(H, e, o);
            for (int r = 0; r < NX; ++r) hess[i * NX * NX + r * NX + j] = o[r];
        }
    }
    return 0;
}
}
