// model.hpp — SE(3) quadrotor model, costs and their derivatives as closed-form device functions.
//
// Reference: quad_model.py:35-119 (Quadrotor.initDyn), :121-213 (initCost / init_TraCost),
// :637-660 (dir_cosine / omega), quad_OC.py:52 (explicit Euler f_d = x + dt f).
// State x = [r(3) v(3) q(4; w,x,y,z) w(3)], control u = 4 rotor thrusts.
//
// Every function works on one lane's registers; the kernels call them either with lane = stage
// (stage-parallel passes) or redundantly on every lane with a broadcast stage (sequential passes).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "lafse3.h"

namespace lafse3 {

constexpr int NX = 13;
constexpr int NU = 4;
constexpr int NA = 17;  // augmented state [x; u_prev]
constexpr int NZ = 21;  // [x~; u]

struct Model {
    double mass, Jx, Jy, Jz, hl, c_tau, grav, dt;
    double ax, ay, az;  // (Jz-Jy)/Jx, (Jx-Jz)/Jy, (Jy-Jx)/Jz
    double wrt, wqt, wthrust, wrf, wvf, wqf, wwf, du_w;
    // reciprocals / products, computed once: an FP64 division is a ~12-instruction dependent sequence on
    // CDNA, and the closed forms below run once per stage in the sequential sweeps.  The oracle uses the
    // same reciprocal forms (oracle/lafse3_oracle.c f_cont / jac_disc / hess_lam_disc).
    double imass, dtm;
    double iJx, iJy, iJz;    // 1/J
    double bwx, bwy, bwz;    // dt*hl/Jx, dt*hl/Jy, dt*c_tau/Jz  (rotor -> angular-rate columns of B)
};

__host__ __host__ __device__ inline Model make_model(const lafse3_params &p)
{
    Model m;
    m.mass = p.mass; m.Jx = p.Jx; m.Jy = p.Jy; m.Jz = p.Jz; m.hl = p.arm_l / 2; m.c_tau = p.c_tau;
    m.grav = p.grav; m.dt = p.dt;
    m.ax = (p.Jz - p.Jy) / p.Jx; m.ay = (p.Jx - p.Jz) / p.Jy; m.az = (p.Jy - p.Jx) / p.Jz;
    m.wrt = p.wrt; m.wqt = p.wqt; m.wthrust = p.wthrust; m.wrf = p.wrf; m.wvf = p.wvf; m.wqf = p.wqf;
    m.wwf = p.wwf; m.du_w = p.du_weight;
    m.imass = 1.0 / p.mass;
    m.dtm = p.dt / p.mass;
    m.iJx = 1.0 / p.Jx; m.iJy = 1.0 / p.Jy; m.iJz = 1.0 / p.Jz;
    m.bwx = p.dt * (p.arm_l / 2) / p.Jx;
    m.bwy = p.dt * (p.arm_l / 2) / p.Jy;
    m.bwz = p.dt * p.c_tau / p.Jz;
    return m;
}

// dir_cosine(q): world -> body (quad_model.py:637-643)
__host__ __device__ inline void dcm(const double *q, double *C)
{
    C[0] = 1 - 2 * (q[2] * q[2] + q[3] * q[3]);
    C[1] = 2 * (q[1] * q[2] + q[0] * q[3]);
    C[2] = 2 * (q[1] * q[3] - q[0] * q[2]);
    C[3] = 2 * (q[1] * q[2] - q[0] * q[3]);
    C[4] = 1 - 2 * (q[1] * q[1] + q[3] * q[3]);
    C[5] = 2 * (q[2] * q[3] + q[0] * q[1]);
    C[6] = 2 * (q[1] * q[3] + q[0] * q[2]);
    C[7] = 2 * (q[2] * q[3] - q[0] * q[1]);
    C[8] = 1 - 2 * (q[1] * q[1] + q[2] * q[2]);
}

// S(Rt) with tr(Rt^T R(q)) = tr(Rt) + q^T S q
__host__ __device__ inline void attitude_form(const double *Rt, double *S)
{
    S[0] = 0;      S[1] = Rt[5] - Rt[7];      S[2] = Rt[6] - Rt[2];       S[3] = Rt[1] - Rt[3];
    S[4] = S[1];   S[5] = -2 * (Rt[4] + Rt[8]); S[6] = Rt[1] + Rt[3];       S[7] = Rt[2] + Rt[6];
    S[8] = S[2];   S[9] = S[6];               S[10] = -2 * (Rt[0] + Rt[8]); S[11] = Rt[5] + Rt[7];
    S[12] = S[3];  S[13] = S[7];              S[14] = S[11];              S[15] = -2 * (Rt[0] + Rt[4]);
}

// continuous dynamics f(x,u) (quad_model.py:86-119)
__host__ __device__ inline void f_cont(const Model &M, const double *x, const double *u, double *f)
{
    const double *v = x + 3, *q = x + 6, *w = x + 10;
    double T = u[0] + u[1] + u[2] + u[3];
    double Mx = -u[1] * M.hl + u[3] * M.hl;
    double My = -u[0] * M.hl + u[2] * M.hl;
    double Mz = (u[0] - u[1] + u[2] - u[3]) * M.c_tau;
    double g0 = 2 * (q[1] * q[3] + q[0] * q[2]);
    double g1 = 2 * (q[2] * q[3] - q[0] * q[1]);
    double g2 = 1 - 2 * (q[1] * q[1] + q[2] * q[2]);
    f[0] = v[0]; f[1] = v[1]; f[2] = v[2];
    const double Tm = T * M.imass;
    f[3] = Tm * g0;
    f[4] = Tm * g1;
    f[5] = Tm * g2 - M.grav;
    f[6] = 0.5 * (-w[0] * q[1] - w[1] * q[2] - w[2] * q[3]);
    f[7] = 0.5 * (w[0] * q[0] + w[2] * q[2] - w[1] * q[3]);
    f[8] = 0.5 * (w[1] * q[0] - w[2] * q[1] + w[0] * q[3]);
    f[9] = 0.5 * (w[2] * q[0] + w[1] * q[1] - w[0] * q[2]);
    f[10] = (Mx - (M.Jz - M.Jy) * w[1] * w[2]) * M.iJx;
    f[11] = (My - (M.Jx - M.Jz) * w[0] * w[2]) * M.iJy;
    f[12] = (Mz - (M.Jy - M.Jx) * w[0] * w[1]) * M.iJz;
}

__host__ __device__ inline void f_disc(const Model &M, const double *x, const double *u, double *xn)
{
    double f[NX];
    f_cont(M, x, u, f);
#pragma unroll
    for (int i = 0; i < NX; ++i) xn[i] = x[i] + M.dt * f[i];
}

// out = A v,  A = d f_d / dx
__host__ __device__ inline void A_times(const Model &M, const double *x, const double *u, const double *v, double *o)
{
    const double *q = x + 6, *w = x + 10;
    const double dt = M.dt;
    double Tm = (u[0] + u[1] + u[2] + u[3]) * M.imass;
    const double *vq = v + 6, *vw = v + 10;
    o[0] = v[0] + dt * v[3];
    o[1] = v[1] + dt * v[4];
    o[2] = v[2] + dt * v[5];
    o[3] = v[3] + dt * Tm * (2 * q[2] * vq[0] + 2 * q[3] * vq[1] + 2 * q[0] * vq[2] + 2 * q[1] * vq[3]);
    o[4] = v[4] + dt * Tm * (-2 * q[1] * vq[0] - 2 * q[0] * vq[1] + 2 * q[3] * vq[2] + 2 * q[2] * vq[3]);
    o[5] = v[5] + dt * Tm * (-4 * q[1] * vq[1] - 4 * q[2] * vq[2]);
    // q rows: (I + dt/2 Omega(w)) vq + dt/2 Xi(q) vw
    o[6] = vq[0] + 0.5 * dt * (-w[0] * vq[1] - w[1] * vq[2] - w[2] * vq[3])
         + 0.5 * dt * (-q[1] * vw[0] - q[2] * vw[1] - q[3] * vw[2]);
    o[7] = vq[1] + 0.5 * dt * (w[0] * vq[0] + w[2] * vq[2] - w[1] * vq[3])
         + 0.5 * dt * (q[0] * vw[0] - q[3] * vw[1] + q[2] * vw[2]);
    o[8] = vq[2] + 0.5 * dt * (w[1] * vq[0] - w[2] * vq[1] + w[0] * vq[3])
         + 0.5 * dt * (q[3] * vw[0] + q[0] * vw[1] - q[1] * vw[2]);
    o[9] = vq[3] + 0.5 * dt * (w[2] * vq[0] + w[1] * vq[1] - w[0] * vq[2])
         + 0.5 * dt * (-q[2] * vw[0] + q[1] * vw[1] + q[0] * vw[2]);
    o[10] = vw[0] - dt * M.ax * (w[2] * vw[1] + w[1] * vw[2]);
    o[11] = vw[1] - dt * M.ay * (w[2] * vw[0] + w[0] * vw[2]);
    o[12] = vw[2] - dt * M.az * (w[1] * vw[0] + w[0] * vw[1]);
}

// out = A^T l
__host__ __device__ inline void At_times(const Model &M, const double *x, const double *u, const double *l, double *o)
{
    const double *q = x + 6, *w = x + 10;
    const double dt = M.dt;
    double Tm = (u[0] + u[1] + u[2] + u[3]) * M.imass;
    const double *lv = l + 3, *lq = l + 6, *lw = l + 10;
    o[0] = l[0]; o[1] = l[1]; o[2] = l[2];
    o[3] = lv[0] + dt * l[0];
    o[4] = lv[1] + dt * l[1];
    o[5] = lv[2] + dt * l[2];
    // q columns: Tm Dg^T lv + 1/2 Omega^T lq
    o[6] = lq[0] + dt * (Tm * (2 * q[2] * lv[0] - 2 * q[1] * lv[1])
                         + 0.5 * (w[0] * lq[1] + w[1] * lq[2] + w[2] * lq[3]));
    o[7] = lq[1] + dt * (Tm * (2 * q[3] * lv[0] - 2 * q[0] * lv[1] - 4 * q[1] * lv[2])
                         + 0.5 * (-w[0] * lq[0] - w[2] * lq[2] + w[1] * lq[3]));
    o[8] = lq[2] + dt * (Tm * (2 * q[0] * lv[0] + 2 * q[3] * lv[1] - 4 * q[2] * lv[2])
                         + 0.5 * (-w[1] * lq[0] + w[2] * lq[1] - w[0] * lq[3]));
    o[9] = lq[3] + dt * (Tm * (2 * q[1] * lv[0] + 2 * q[2] * lv[1])
                         + 0.5 * (-w[2] * lq[0] - w[1] * lq[1] + w[0] * lq[2]));
    // w columns: 1/2 Xi^T lq + Jw^T lw
    o[10] = lw[0] + dt * (0.5 * (-q[1] * lq[0] + q[0] * lq[1] + q[3] * lq[2] - q[2] * lq[3])
                          - M.ay * w[2] * lw[1] - M.az * w[1] * lw[2]);
    o[11] = lw[1] + dt * (0.5 * (-q[2] * lq[0] - q[3] * lq[1] + q[0] * lq[2] + q[1] * lq[3])
                          - M.ax * w[2] * lw[0] - M.az * w[0] * lw[2]);
    o[12] = lw[2] + dt * (0.5 * (-q[3] * lq[0] + q[2] * lq[1] - q[1] * lq[2] + q[0] * lq[3])
                          - M.ax * w[1] * lw[0] - M.ay * w[0] * lw[1]);
}

// rotor-to-angular-acceleration matrix row d, column a: dt * M_w[d][a]
__host__ __device__ inline double Bw(const Model &M, int d, int a)
{
    if (d == 0) return (a == 1) ? -M.bwx : (a == 3 ? M.bwx : 0.0);
    if (d == 1) return (a == 0) ? -M.bwy : (a == 2 ? M.bwy : 0.0);
    return ((a & 1) ? -1.0 : 1.0) * M.bwz;
}

// out = B du  (B = d f_d / du)
__host__ __device__ inline void B_times(const Model &M, const double *x, const double *du, double *o)
{
    const double *q = x + 6;
        double s = du[0] + du[1] + du[2] + du[3];
    double g0 = 2 * (q[1] * q[3] + q[0] * q[2]);
    double g1 = 2 * (q[2] * q[3] - q[0] * q[1]);
    double g2 = 1 - 2 * (q[1] * q[1] + q[2] * q[2]);
#pragma unroll
    for (int i = 0; i < NX; ++i) o[i] = 0.0;
    o[3] = M.dtm * g0 * s;
    o[4] = M.dtm * g1 * s;
    o[5] = M.dtm * g2 * s;
    o[10] = M.bwx * (du[3] - du[1]);
    o[11] = M.bwy * (du[2] - du[0]);
    o[12] = M.bwz * (du[0] - du[1] + du[2] - du[3]);
}

// out = B^T l
__host__ __device__ inline void Bt_times(const Model &M, const double *x, const double *l, double *o)
{
    const double *q = x + 6;
        double g0 = 2 * (q[1] * q[3] + q[0] * q[2]);
    double g1 = 2 * (q[2] * q[3] - q[0] * q[1]);
    double g2 = 1 - 2 * (q[1] * q[1] + q[2] * q[2]);
    double v = M.dtm * (g0 * l[3] + g1 * l[4] + g2 * l[5]);
    double ex = M.bwx * l[10], ey = M.bwy * l[11], ez = M.bwz * l[12];
    o[0] = v - ey + ez;
    o[1] = v - ex - ez;
    o[2] = v + ey + ez;
    o[3] = v + ex - ez;
}

// per-instance attitude data (the 4x4 forms live in LDS; only pointers travel in registers)
struct Attitude {
    double St[16];     // traversal: tau = 3 - trRt - q^T St q
    double Sg[16];     // goal attitude (weight wqf)
    double trRt, trRg;
};

// tau = trace(I - Rt^T R(q)) evaluated as in quad_model.py:210
__host__ __device__ inline double att_tau(const double *St, double trR, const double *q)
{
    double s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double a = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) a += St[i * 4 + j] * q[j];
        s += q[i] * a;
    }
    return 3.0 - trR - s;
}

// wk*tra(x) + path(x)  (quad_model.py:191-213)
__host__ __device__ inline double state_cost(const Model &M, const Attitude &at, const double *goal, const double *ptra,
                                    double wk, const double *x)
{
    double er = 0, ev = 0, ew = 0, et = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double d = x[i] - goal[i];
        er += d * d;
        ev += x[3 + i] * x[3 + i];
        ew += x[10 + i] * x[10 + i];
        double e = x[i] - ptra[i];
        et += e * e;
    }
    double c = M.wrf * er + M.wvf * ev + M.wwf * ew;
    if (M.wqf != 0.0) c += M.wqf * att_tau(at.Sg, at.trRg, x + 6);
    if (wk != 0.0) {
        double tau = att_tau(at.St, at.trRt, x + 6);
        c += wk * (M.wrt * et + M.wqt * tau * tau);
    }
    return c;
}

// gradient of wk*tra + path at x (13)
__host__ __device__ inline void state_cost_grad(const Model &M, const Attitude &at, const double *goal, const double *ptra,
                                       double wk, const double *x, double *g)
{
    const double *q = x + 6;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        g[i] = 2 * M.wrf * (x[i] - goal[i]) + wk * 2 * M.wrt * (x[i] - ptra[i]);
        g[3 + i] = 2 * M.wvf * x[3 + i];
        g[10 + i] = 2 * M.wwf * x[10 + i];
    }
    double Sq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double a = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) a += at.St[i * 4 + j] * q[j];
        Sq[i] = a;
    }
    double tau = att_tau(at.St, at.trRt, q);
    double cw = wk * M.wqt;
#pragma unroll
    for (int i = 0; i < 4; ++i) g[6 + i] = cw * 2 * tau * (-2 * Sq[i]);
    if (M.wqf != 0.0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double a = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) a += at.Sg[i * 4 + j] * q[j];
            g[6 + i] += M.wqf * (-2 * a);
        }
    }
}

// Stage Hessian pieces that the Riccati needs, computed once per stage from (x_k, u_k, lam_k):
//   cost part (times s):  Hc_r = 2(wrf + wk wrt), Hc_v = 2 wvf, Hc_w = 2 wwf, Hc_qq (4x4)
//   constraint part:      Hl_qq (4x4), Hl_qw (4x3), Hl_ww off-diagonals, Hl_qu (4, same for every rotor)
struct StageHess {
    double hr, hv, hw;        // diagonal (already scaled by s)
    double qq[16];            // q-q block (cost*s + lambda part)
    double qw[12];            // q-w block (lambda part), row q_i col w_c
    double wyz, wxz, wxy;     // w-w off-diagonals (lambda part)
    double qu[4];             // q-u coupling, same for each rotor
};

__host__ __device__ inline void stage_hessian(const Model &M, const Attitude &at, double s, double wk, const double *x,
                                     const double *u, const double *lam, StageHess &H)
{
    const double *q = x + 6;
    const double dt = M.dt;
    double Tm = (u[0] + u[1] + u[2] + u[3]) * M.imass;
    H.hr = s * 2 * (M.wrf + wk * M.wrt);
    H.hv = s * 2 * M.wvf;
    H.hw = s * 2 * M.wwf;
    double Sq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double a = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) a += at.St[i * 4 + j] * q[j];
        Sq[i] = a;
    }
    double tau = att_tau(at.St, at.trRt, q);
    double cw = s * wk * M.wqt;
    double a0 = lam[3], a1 = lam[4], a2 = lam[5];
    const double Hq[16] = {0, -2 * a1, 2 * a0, 0,
                           -2 * a1, -4 * a2, 0, 2 * a0,
                           2 * a0, 0, -4 * a2, 2 * a1,
                           0, 2 * a0, 2 * a1, 0};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double h = cw * (8 * Sq[i] * Sq[j] - 4 * tau * at.St[i * 4 + j]) + dt * Tm * Hq[i * 4 + j];
            if (M.wqf != 0.0) h += s * M.wqf * (-2 * at.Sg[i * 4 + j]);
            H.qq[i * 4 + j] = h;
        }
    double m0 = lam[6], m1 = lam[7], m2 = lam[8], m3 = lam[9];
    const double Hqw[12] = {m1, m2, m3,
                            -m0, m3, -m2,
                            -m3, -m0, m1,
                            m2, -m1, -m0};
#pragma unroll
    for (int i = 0; i < 12; ++i) H.qw[i] = dt * 0.5 * Hqw[i];
    H.wyz = -dt * lam[10] * M.ax;
    H.wxz = -dt * lam[11] * M.ay;
    H.wxy = -dt * lam[12] * M.az;
    H.qu[0] = M.dtm * (2 * a0 * q[2] - 2 * a1 * q[1]);
    H.qu[1] = M.dtm * (2 * a0 * q[3] - 2 * a1 * q[0] - 4 * a2 * q[1]);
    H.qu[2] = M.dtm * (2 * a0 * q[0] + 2 * a1 * q[3] - 4 * a2 * q[2]);
    H.qu[3] = M.dtm * (2 * a0 * q[1] + 2 * a1 * q[2]);
}

// o = Hxx v (x-x block of the stage Hessian, without Sigma / delta_w)
__host__ __device__ inline void Hxx_times(const StageHess &H, const double *v, double *o)
{
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        o[i] = H.hr * v[i];
        o[3 + i] = H.hv * v[3 + i];
        o[10 + i] = H.hw * v[10 + i];
    }
    const double *vq = v + 6, *vw = v + 10;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double a = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) a += H.qq[i * 4 + j] * vq[j];
#pragma unroll
        for (int c = 0; c < 3; ++c) a += H.qw[i * 3 + c] * vw[c];
        o[6 + i] = a;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double a = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) a += H.qw[i * 3 + c] * vq[i];
        o[10 + c] += a;
    }
    o[10] += H.wxy * vw[1] + H.wxz * vw[2];
    o[11] += H.wxy * vw[0] + H.wyz * vw[2];
    o[12] += H.wxz * vw[0] + H.wyz * vw[1];
}

}  // namespace lafse3
