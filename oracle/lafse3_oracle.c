/*
 * lafse3_oracle.c — TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).
 *
 * Plain-C, fp64, scalar restatement of the reference's optimal-control hot path
 * (yanrui89/LearningAgileFlight_SE3 @ 2025-01-24):
 *
 *   model      quad_model.py:35-119   (Quadrotor.initDyn: SE(3) rigid body, quaternion, 4 rotors)
 *              quad_model.py:637-660  (dir_cosine / skew / omega)
 *   costs      quad_model.py:121-213  (initCost / init_TraCost), weights quad_policy.py:37-38
 *   NLP        quad_OC.py:104-212     (OCSys.ocSolver: multiple shooting, Euler f_d, IPOPT defaults)
 *              bounds quad_policy.py:46-51, dt quad_policy.py:43
 *   reward     quad_policy.py:67-91   (run_quad.objective), quad_model.py:239-276 (rotor tips),
 *              solid_geometry.py:7-168 (plane / line / obstacle.collis_det)
 *   gradient   quad_policy.py:94-112  (run_quad.sol_gradient, 9-solve clipped forward difference)
 *   t / angle  quad_policy.py:10-13 (Rd2Rp), quad_model.py:818-825 (toQuaternion)
 *
 * The reference solves the NLP with CasADi 3.5.5 + IPOPT (MUMPS) — neither exists in this image,
 * so the NLP optimum itself is NOT pinned by any reference run: this file restates the same NLP
 * and solves it with an IPOPT-style primal-dual barrier method (Waechter & Biegler 2006 defaults:
 * mu_init 0.1, monotone mu, tau_min 0.99, filter line search, inertia correction, kappa_sigma
 * safeguard, gradient-based objective scaling, least-squares constraint multipliers, bound
 * relaxation 1e-8, tol 1e-8) whose KKT system is solved by a Riccati recursion on the state
 * augmented with the previous control (the ||U_k - U_{k-1}||^2 term couples stages).
 * Its optima are certified by an independent torch-autograd restatement of the NLP (tests/kkt.py):
 * tests/test_oracle_golden.py::test_policy_fixture_optima_are_kkt_points (the fixture's optima),
 * ::test_oracle_optimum_matches_trust_constr (scipy trust-constr on the same NLP, a solver sharing no
 * code with this file) and tests/test_gpu_parity.py::test_ocp_solve_matches_oracle_and_is_kkt.
 * The IFT gradient mode (orc_ift_probes) is pinned by the GPU tests against this file only.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * The product path (learningagileflight_se3_amd/) never links or calls it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#if defined(ORC_TRACE) || defined(ORC_RTRACE)
#include <stdio.h>
#endif
#ifdef _OPENMP
#include <omp.h>
#endif

#define NX 13
#define NU 4
#define NA 17          /* augmented state [x; u_prev] */
#define NMAX 64
#define FILTER_MAX 64
#define NMAX_DUMP 50

typedef struct {
    /* model (quad_policy.py:37, quad_model.py:37) */
    double mass, Jx, Jy, Jz, arm_l, c_tau, grav, dt;
    /* cost weights (quad_policy.py:38, quad_OC.py:145,150) */
    double wrt, wqt, wthrust, wrf, wvf, wqf, wwf;
    double tra_w_peak, tra_w_decay, du_weight;
    /* bounds (quad_policy.py:46-51) */
    double u_lb, u_ub, w_lb, w_ub;
    /* reward (quad_policy.py:19, solid_geometry.py:115) */
    double wing_len, d_min;
    int32_t horizon;
    /* IPOPT options (defaults of IPOPT 3.12 as shipped with casadi 3.5.5) */
    int32_t max_iter;
    double tol, acceptable_tol;
    int32_t acceptable_iter;
    double mu_init, bound_relax;
    int32_t lsq_mult_init;
    /* 1: NumPy >= 2 (NEP 50) scalar promotion in sol_gradient — the t+-0.1 probes and the
     * 1/(500 a^2 + 5) factors stay float32 — instead of the float64 of the reference environment
     * (NumPy 1.23, README.md:23).  Used only to compare against golden vectors made in this image. */
    int32_t t_probe_f32;
    /* IPOPT max_soc (default 4): second-order corrections tried on a rejected first trial point */
    int32_t max_soc;
    /* 1: IPOPT's restoration phase when the line search and the soft restoration phase fail (default); 0: the
     * solve ends there (status 3, round 2's behaviour) */
    int32_t restoration;
    /* IPOPT watchdog_shortened_iter_trigger (default 10; 0 disables): after this many successive iterations whose
     * line search rejected the first trial point, up to watchdog_trial_iter_max (3) full steps are taken without
     * the line search before the stored iterate is resumed (BacktrackingLineSearch watchdog procedure) */
    int32_t watchdog;
    /* sol_gradient gradient mode (lafse3_params.grad_mode): 0 = the reference's 9-solve finite differences
     * (quad_policy.py:94-112); 1 = implicit-function sensitivities of the nominal optimum for the six
     * p_tra / a_tra probes (orc_ift_probes), the t probes still solved */
    int32_t grad_mode;
} orc_params;

typedef struct {
    double ini[NX];
    double goal[3];
    double ptra[3];
    double qtra[4];
    double t;         /* traversal time used in the stage weight (already rounded by caller) */
    double ulast[4];
} orc_inst;

enum { ST_SOLVED = 0, ST_ACCEPTABLE = 1, ST_MAXITER = 2, ST_LS_FAIL = 3, ST_NONFINITE = 4,
       ST_TINY = 5, ST_REG_FAIL = 6 };   /* 8 ST_RESTO_FAIL, 9 ST_INFEASIBLE: restoration phase (below) */

/* ------------------------------------------------------------------------------------------ */
/* model                                                                                       */
/* ------------------------------------------------------------------------------------------ */

/* dir_cosine(q): quad_model.py:637-643 (world -> body) */
static void dir_cosine(const double *q, double *C)
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

/* continuous dynamics f(x,u): quad_model.py:86-119 */
static void f_cont(const orc_params *P, const double *x, const double *u, double *f)
{
    const double *v = x + 3, *q = x + 6, *w = x + 10;
    double T = u[0] + u[1] + u[2] + u[3];
    double Mx = -u[1] * P->arm_l / 2 + u[3] * P->arm_l / 2;
    double My = -u[0] * P->arm_l / 2 + u[2] * P->arm_l / 2;
    double Mz = (u[0] - u[1] + u[2] - u[3]) * P->c_tau;
    double C[9];
    dir_cosine(q, C);
    /* dv = (1/m) C^T [0,0,T] + g_I  — C^T e3 is the third row of C */
    f[0] = v[0]; f[1] = v[1]; f[2] = v[2];
    /* reciprocal forms (x * (1/m) rather than x / m), as the device closed forms (model.hpp) */
    const double Tm = T * (1.0 / P->mass);
    f[3] = Tm * C[6];
    f[4] = Tm * C[7];
    f[5] = Tm * C[8] - P->grav;
    /* dq = 1/2 Omega(w) q */
    f[6] = 0.5 * (-w[0] * q[1] - w[1] * q[2] - w[2] * q[3]);
    f[7] = 0.5 * (w[0] * q[0] + w[2] * q[2] - w[1] * q[3]);
    f[8] = 0.5 * (w[1] * q[0] - w[2] * q[1] + w[0] * q[3]);
    f[9] = 0.5 * (w[2] * q[0] + w[1] * q[1] - w[0] * q[2]);
    /* dw = J^-1 (M - w x (J w)) */
    f[10] = (Mx - (P->Jz - P->Jy) * w[1] * w[2]) * (1.0 / P->Jx);
    f[11] = (My - (P->Jx - P->Jz) * w[0] * w[2]) * (1.0 / P->Jy);
    f[12] = (Mz - (P->Jy - P->Jx) * w[0] * w[1]) * (1.0 / P->Jz);
}

/* f_d = x + dt f: quad_OC.py:52 */
static void f_disc(const orc_params *P, const double *x, const double *u, double *xn)
{
    double f[NX];
    f_cont(P, x, u, f);
    for (int i = 0; i < NX; ++i) xn[i] = x[i] + P->dt * f[i];
}

/* A = d f_d / dx (13x13 row-major), B = d f_d / du (13x4) */
static void jac_disc(const orc_params *P, const double *x, const double *u, double *A, double *B)
{
    const double *q = x + 6, *w = x + 10;
    const double dt = P->dt;
    double T = u[0] + u[1] + u[2] + u[3];
    double Tm = T * (1.0 / P->mass);
    memset(A, 0, sizeof(double) * NX * NX);
    memset(B, 0, sizeof(double) * NX * NU);
    for (int i = 0; i < NX; ++i) A[i * NX + i] = 1.0;
    for (int i = 0; i < 3; ++i) A[i * NX + 3 + i] += dt;
    /* v rows */
    double dg0[4] = {2 * q[2], 2 * q[3], 2 * q[0], 2 * q[1]};
    double dg1[4] = {-2 * q[1], -2 * q[0], 2 * q[3], 2 * q[2]};
    double dg2[4] = {0, -4 * q[1], -4 * q[2], 0};
    for (int j = 0; j < 4; ++j) {
        A[3 * NX + 6 + j] += dt * Tm * dg0[j];
        A[4 * NX + 6 + j] += dt * Tm * dg1[j];
        A[5 * NX + 6 + j] += dt * Tm * dg2[j];
    }
    double C[9];
    dir_cosine(q, C);
    for (int j = 0; j < 4; ++j) {
        B[3 * NU + j] = (dt / P->mass) * C[6];
        B[4 * NU + j] = (dt / P->mass) * C[7];
        B[5 * NU + j] = (dt / P->mass) * C[8];
    }
    /* q rows: dq/dq = 1/2 Omega(w), dq/dw */
    double Om[16] = {0, -w[0], -w[1], -w[2],
                     w[0], 0, w[2], -w[1],
                     w[1], -w[2], 0, w[0],
                     w[2], w[1], -w[0], 0};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) A[(6 + i) * NX + 6 + j] += dt * 0.5 * Om[i * 4 + j];
    double Xi[12] = {-q[1], -q[2], -q[3],
                     q[0], -q[3], q[2],
                     q[3], q[0], -q[1],
                     -q[2], q[1], q[0]};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j) A[(6 + i) * NX + 10 + j] += dt * 0.5 * Xi[i * 3 + j];
    /* w rows */
    double ax = (P->Jz - P->Jy) / P->Jx, ay = (P->Jx - P->Jz) / P->Jy, az = (P->Jy - P->Jx) / P->Jz;
    A[10 * NX + 11] += -dt * ax * w[2];
    A[10 * NX + 12] += -dt * ax * w[1];
    A[11 * NX + 10] += -dt * ay * w[2];
    A[11 * NX + 12] += -dt * ay * w[0];
    A[12 * NX + 10] += -dt * az * w[1];
    A[12 * NX + 11] += -dt * az * w[0];
    double hl = P->arm_l / 2;
    B[10 * NU + 1] = -(dt * hl / P->Jx); B[10 * NU + 3] = dt * hl / P->Jx;
    B[11 * NU + 0] = -(dt * hl / P->Jy); B[11 * NU + 2] = dt * hl / P->Jy;
    B[12 * NU + 0] = dt * P->c_tau / P->Jz; B[12 * NU + 1] = -(dt * P->c_tau / P->Jz);
    B[12 * NU + 2] = dt * P->c_tau / P->Jz; B[12 * NU + 3] = -(dt * P->c_tau / P->Jz);
}

/* Hxx += sum_i lam_i d2 f_d,i/dx2 ; Hxu += sum_i lam_i d2 f_d,i/dxdu  (Huu contribution is 0) */
static void hess_lam_disc(const orc_params *P, const double *x, const double *u, const double *lam,
                          double *Hxx, double *Hxu)
{
    const double *q = x + 6;
    const double dt = P->dt;
    double T = u[0] + u[1] + u[2] + u[3];
    double Tm = T * (1.0 / P->mass);
    double a0 = lam[3], a1 = lam[4], a2 = lam[5];
    /* q-q from v rows */
    double Hq[16] = {0, -2 * a1, 2 * a0, 0,
                     -2 * a1, -4 * a2, 0, 2 * a0,
                     2 * a0, 0, -4 * a2, 2 * a1,
                     0, 2 * a0, 2 * a1, 0};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) Hxx[(6 + i) * NX + 6 + j] += dt * Tm * Hq[i * 4 + j];
    /* q-u from v rows: (1/m) grad_q (a . g(q)) for every rotor */
    double gq[4] = {2 * a0 * q[2] - 2 * a1 * q[1],
                    2 * a0 * q[3] - 2 * a1 * q[0] - 4 * a2 * q[1],
                    2 * a0 * q[0] + 2 * a1 * q[3] - 4 * a2 * q[2],
                    2 * a0 * q[1] + 2 * a1 * q[2]};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < NU; ++j) Hxu[(6 + i) * NU + j] += (dt / P->mass) * gq[i];
    /* q-w from q rows */
    double m0 = lam[6], m1 = lam[7], m2 = lam[8], m3 = lam[9];
    double Hqw[12] = {m1, m2, m3,
                      -m0, m3, -m2,
                      -m3, -m0, m1,
                      m2, -m1, -m0};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j) {
            double h = dt * 0.5 * Hqw[i * 3 + j];
            Hxx[(6 + i) * NX + 10 + j] += h;
            Hxx[(10 + j) * NX + 6 + i] += h;
        }
    /* w-w from w rows */
    double ax = (P->Jz - P->Jy) / P->Jx, ay = (P->Jx - P->Jz) / P->Jy, az = (P->Jy - P->Jx) / P->Jz;
    double hyz = -dt * lam[10] * ax, hxz = -dt * lam[11] * ay, hxy = -dt * lam[12] * az;
    Hxx[11 * NX + 12] += hyz; Hxx[12 * NX + 11] += hyz;
    Hxx[10 * NX + 12] += hxz; Hxx[12 * NX + 10] += hxz;
    Hxx[10 * NX + 11] += hxy; Hxx[11 * NX + 10] += hxy;
}

/* S(Rt): tr(Rt^T R(q)) = tr(Rt) + q^T S q  (quadratic form of dir_cosine) */
static void attitude_form(const double *Rt, double *S)
{
    S[0] = 0;                       S[1] = Rt[5] - Rt[7];          S[2] = Rt[6] - Rt[2];          S[3] = Rt[1] - Rt[3];
    S[4] = S[1];                    S[5] = -2 * (Rt[4] + Rt[8]);    S[6] = Rt[1] + Rt[3];          S[7] = Rt[2] + Rt[6];
    S[8] = S[2];                    S[9] = S[6];                   S[10] = -2 * (Rt[0] + Rt[8]);   S[11] = Rt[5] + Rt[7];
    S[12] = S[3];                   S[13] = S[7];                  S[14] = S[11];                 S[15] = -2 * (Rt[0] + Rt[4]);
}

typedef struct {
    double Rt[9], St[16];  /* traversal attitude */
    double Rg[9], Sg[16];  /* goal attitude (weight wqf) */
} att_t;

/* tau = trace(I - Rt^T R(q))  (quad_model.py:178, :210) */
static double att_trace(const double *Rt, const double *q)
{
    double R[9];
    dir_cosine(q, R);
    double s = 0;
    for (int i = 0; i < 9; ++i) s += Rt[i] * R[i];
    return 3.0 - s;
}

/* path / final cost (quad_model.py:191-198) */
static double path_cost(const orc_params *P, const att_t *at, const double *goal, const double *x)
{
    double er = 0, ev = 0, ew = 0;
    for (int i = 0; i < 3; ++i) {
        double d = x[i] - goal[i];
        er += d * d;
        ev += x[3 + i] * x[3 + i];
        ew += x[10 + i] * x[10 + i];
    }
    double c = P->wrf * er + P->wvf * ev + P->wwf * ew;
    if (P->wqf != 0.0) c += P->wqf * att_trace(at->Rg, x + 6);
    return c;
}

/* traversal cost (quad_model.py:200-213) */
static double tra_cost(const orc_params *P, const att_t *at, const double *ptra, const double *x)
{
    double er = 0;
    for (int i = 0; i < 3; ++i) {
        double d = x[i] - ptra[i];
        er += d * d;
    }
    double tau = att_trace(at->Rt, x + 6);
    return P->wrt * er + P->wqt * tau * tau;
}

/* stage weight w_k = 60 exp(-10 (dt k - t)^2)  (quad_OC.py:145) */
static double stage_weight(const orc_params *P, int k, double t)
{
    double d = P->dt * k - t;
    return P->tra_w_peak * exp(-P->tra_w_decay * d * d);
}

/* gradient (13) and Hessian (13x13, += ) of  wk*tra + path  at x */
static void state_cost_derivs(const orc_params *P, const att_t *at, const double *goal,
                              const double *ptra, double wk, const double *x, double *g, double *H)
{
    const double *q = x + 6;
    memset(g, 0, sizeof(double) * NX);
    for (int i = 0; i < 3; ++i) {
        g[i] = 2 * P->wrf * (x[i] - goal[i]) + wk * 2 * P->wrt * (x[i] - ptra[i]);
        g[3 + i] = 2 * P->wvf * x[3 + i];
        g[10 + i] = 2 * P->wwf * x[10 + i];
        if (H) {
            H[i * NX + i] += 2 * P->wrf + wk * 2 * P->wrt;
            H[(3 + i) * NX + 3 + i] += 2 * P->wvf;
            H[(10 + i) * NX + 10 + i] += 2 * P->wwf;
        }
    }
    /* traversal attitude: wk*wqt*tau^2, tau = 3 - tr(Rt) - q^T St q */
    double Sq[4];
    for (int i = 0; i < 4; ++i) {
        Sq[i] = 0;
        for (int j = 0; j < 4; ++j) Sq[i] += at->St[i * 4 + j] * q[j];
    }
    double tau = att_trace(at->Rt, q);
    double cw = wk * P->wqt;
    for (int i = 0; i < 4; ++i) g[6 + i] += cw * 2 * tau * (-2 * Sq[i]);
    if (H)
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                H[(6 + i) * NX + 6 + j] += cw * (8 * Sq[i] * Sq[j] - 4 * tau * at->St[i * 4 + j]);
    if (P->wqf != 0.0) {
        double Sg[4];
        for (int i = 0; i < 4; ++i) {
            Sg[i] = 0;
            for (int j = 0; j < 4; ++j) Sg[i] += at->Sg[i * 4 + j] * q[j];
        }
        for (int i = 0; i < 4; ++i) g[6 + i] += P->wqf * (-2 * Sg[i]);
        if (H)
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) H[(6 + i) * NX + 6 + j] += P->wqf * (-2 * at->Sg[i * 4 + j]);
    }
}

static double dot3(const double *a, const double *b);
static double magni3(const double *v);

/* toQuaternion(angle, dir)  quad_model.py:818-825 */
static void to_quaternion(double angle, const double *dir, double *q)
{
    double n = magni3(dir);  /* numpy.linalg.norm(dir) = sqrt(dot(dir, dir)) */
    q[0] = cos(angle / 2);
    double s = sin(angle / 2);
    q[1] = s * (dir[0] / n);
    q[2] = s * (dir[1] / n);
    q[3] = s * (dir[2] / n);
}

/* Rd2Rp (quad_policy.py:10-13) + toQuaternion; a_norm = magni(tra_ang) supplied by the caller
 * (fp32 or fp64 depending on the dtype the reference saw) */
void orc_rd2quat(double a_norm, const double *a, double *q)
{
    double theta = 2.0 * atan(a_norm);
    double v[3] = {a[0] + 1e-8, a[1], a[2]};
    double m = magni3(v);    /* norm(): solid_geometry.py:11-12 */
    double n[3] = {v[0] / m, v[1] / m, v[2] / m};
    to_quaternion(theta, n, q);
}

/* ------------------------------------------------------------------------------------------ */
/* dense helpers                                                                               */
/* ------------------------------------------------------------------------------------------ */

/* Cholesky of a 4x4 SPD block.  The diagonal is used through its reciprocals (stored in the unused
 * upper triangle: L[j*4+3-...] would be awkward, so a separate array rides along in L[16..19]); the
 * device kernels follow the same operation order so both sides take the same IPM decisions. */
static int chol4(const double *M, double *L)
{
    /* M 4x4 SPD -> lower L (row-major) + L[16+j] = 1/L[j][j]; returns 0 on success */
    memset(L, 0, sizeof(double) * 20);
    for (int j = 0; j < 4; ++j) {
        double d = M[j * 4 + j];
        for (int k = 0; k < j; ++k) d -= L[j * 4 + k] * L[j * 4 + k];
        if (!(d > 0.0)) return -1;
        double ljj = sqrt(d);
        L[j * 4 + j] = ljj;
        L[16 + j] = 1.0 / ljj;
        for (int i = j + 1; i < 4; ++i) {
            double s = M[i * 4 + j];
            for (int k = 0; k < j; ++k) s -= L[i * 4 + k] * L[j * 4 + k];
            L[i * 4 + j] = s * L[16 + j];
        }
    }
    return 0;
}

static void chol4_solve(const double *L, double *b)
{
    for (int i = 0; i < 4; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * 4 + k] * b[k];
        b[i] = s * L[16 + i];
    }
    for (int i = 3; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < 4; ++k) s -= L[k * 4 + i] * b[k];
        b[i] = s * L[16 + i];
    }
}

/* ------------------------------------------------------------------------------------------ */
/* IPM workspace                                                                               */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    int N;
    double s_obj;                       /* objective scaling */
    double x[(NMAX + 1) * NX], u[NMAX * NU], lam[NMAX * NX];
    double zLu[NMAX * NU], zUu[NMAX * NU], zLw[(NMAX + 1) * 3], zUw[(NMAX + 1) * 3];
    double dx[(NMAX + 1) * NX], du[NMAX * NU], lamp[NMAX * NX];
    double K[NMAX * NU * NA], kff[NMAX * NU];
    /* iterative refinement: when refine != 0 the stage right-hand sides are taken from these */
    int refine;
    double rq[(NMAX + 1) * NX], rr[NMAX * NU], rc[NMAX * NX];
    /* second-order correction: when soc != 0 the (non-refinement) stage constraint part is cs */
    int soc;
    double cs[NMAX * NX];
    double wk[NMAX + 1];
    double ulo, uhi, wlo, whi;          /* relaxed bounds */
    att_t at;
    /* counters */
    int iters, sweeps, trials, refines, socs, restos;
    double mu;
    double *trace;     /* debug: 16 doubles per iteration (nullable) */
    double mJ, mlb;    /* debug: objective J and barrier log sum of the last eval_merit */
    int trace_iters;
    double *dump;      /* debug: Newton step of iteration dump_it */
    int dump_it, dump_refine;
    /* optimality error at the last iterate (IPOPT's "Overall NLP error" and its unscaled parts) */
    double fin_err, fin_dual, fin_primal, fin_compl;
} orc_ws;

/* barrier gradient & Sigma for a box-bounded scalar */
static inline void bar_terms(double v, double lo, double hi, double zl, double zu, double mu,
                             double *grad, double *sig)
{
    double sl = v - lo, su = hi - v;
    *grad = -mu / sl + mu / su;
    *sig = zl / sl + zu / su;
}

/* gradient of the scaled objective w.r.t. x_k (k>=1) — without barrier */
static void grad_x(const orc_params *P, const orc_inst *I, orc_ws *W, int k, double *g)
{
    double w = (k < W->N) ? W->wk[k] : 0.0;
    state_cost_derivs(P, &W->at, I->goal, I->ptra, w, W->x + k * NX, g, NULL);
    for (int i = 0; i < NX; ++i) g[i] *= W->s_obj;
}

/* gradient of the scaled objective w.r.t. u_k — without barrier */
static void grad_u(const orc_params *P, const orc_inst *I, orc_ws *W, int k, double *g)
{
    const double *uk = W->u + k * NU;
    const double *up = (k == 0) ? I->ulast : W->u + (k - 1) * NU;
    for (int j = 0; j < NU; ++j) {
        g[j] = 2 * P->wthrust * uk[j] + P->du_weight * 2 * (uk[j] - up[j]);
        if (k + 1 < W->N) g[j] += -P->du_weight * 2 * (W->u[(k + 1) * NU + j] - uk[j]);
        g[j] *= W->s_obj;
    }
}

/* objective J (unscaled) at arbitrary trajectories */
static double objective_J(const orc_params *P, const orc_inst *I, orc_ws *W, const double *x, const double *u)
{
    double J = 0;
    for (int k = 0; k < W->N; ++k) {
        const double *xk = x + k * NX, *uk = u + k * NU;
        const double *up = (k == 0) ? I->ulast : u + (k - 1) * NU;
        double c = W->wk[k] * tra_cost(P, &W->at, I->ptra, xk) + path_cost(P, &W->at, I->goal, xk);
        double th = 0, sm = 0;
        for (int j = 0; j < NU; ++j) {
            th += uk[j] * uk[j];
            sm += (uk[j] - up[j]) * (uk[j] - up[j]);
        }
        c += P->wthrust * th + P->du_weight * sm;
        J += c;
    }
    J += path_cost(P, &W->at, I->goal, x + W->N * NX);
    return J;
}

/* theta = ||c||_1 and barrier objective phi at (x,u) */
static void eval_merit(const orc_params *P, const orc_inst *I, orc_ws *W, const double *x, const double *u,
                       double mu, double *theta, double *phi, int *ok)
{
    double th = 0, lb = 0;
    int good = 1;
    for (int k = 0; k < W->N; ++k) {
        double xn[NX];
        f_disc(P, x + k * NX, u + k * NU, xn);
        for (int i = 0; i < NX; ++i) th += fabs(xn[i] - x[(k + 1) * NX + i]);
        for (int j = 0; j < NU; ++j) {
            double v = u[k * NU + j];
            double sl = v - W->ulo, su = W->uhi - v;
            if (!(sl > 0) || !(su > 0)) good = 0;
            lb += log(sl) + log(su);
        }
    }
    for (int k = 1; k <= W->N; ++k)
        for (int j = 0; j < 3; ++j) {
            double v = x[k * NX + 10 + j];
            double sl = v - W->wlo, su = W->whi - v;
            if (!(sl > 0) || !(su > 0)) good = 0;
            lb += log(sl) + log(su);
        }
    double J = objective_J(P, I, W, x, u);
    W->mJ = J;
    W->mlb = lb;
    *theta = th;
    *phi = W->s_obj * J - mu * lb;
    *ok = good && isfinite(*phi) && isfinite(th);
}

/* ---- stage QP data ---------------------------------------------------------------------- */
/* For stage k (0..N-1): augmented x~ = [x_k; u_{k-1}], control u_k.
 *  Q (17x17), S (17x4), R (4x4), q (17), r (4), A~ (17x17 with only [0:13,0:13] = A), B~ = [B; I],
 *  c~ = [f_d(x_k,u_k) - x_{k+1}; 0]. mode_lsq: Hessian replaced by identity (LS multipliers). */
typedef struct {
    double Q[NA * NA], S[NA * NU], R[NU * NU], q[NA], r[NU];
    double A[NX * NX], B[NX * NU], c[NX];
} stage_qp;

static void build_stage(const orc_params *P, const orc_inst *I, orc_ws *W, int k, double delta_w,
                        int mode_lsq, stage_qp *sq)
{
    const double *xk = W->x + k * NX, *uk = W->u + k * NU;
    memset(sq, 0, sizeof(*sq));
    jac_disc(P, xk, uk, sq->A, sq->B);
    double xn[NX];
    f_disc(P, xk, uk, xn);
    for (int i = 0; i < NX; ++i) sq->c[i] = mode_lsq ? 0.0 : (W->soc ? W->cs[k * NX + i] : xn[i] - W->x[(k + 1) * NX + i]);
    const double s = W->s_obj;
    double Hxx[NX * NX], Hxu[NX * NU];
    memset(Hxx, 0, sizeof(Hxx));
    memset(Hxu, 0, sizeof(Hxu));
    double gx[NX];
    if (k >= 1) {
        state_cost_derivs(P, &W->at, I->goal, I->ptra, W->wk[k], xk, gx, mode_lsq ? NULL : Hxx);
        for (int i = 0; i < NX; ++i) gx[i] *= s;
        if (!mode_lsq) {
            for (int i = 0; i < NX * NX; ++i) Hxx[i] *= s;
            hess_lam_disc(P, xk, uk, W->lam + k * NX, Hxx, Hxu);
        }
    }
    /* x block */
    if (k >= 1) {
        for (int i = 0; i < NX; ++i)
            for (int j = 0; j < NX; ++j) sq->Q[i * NA + j] = Hxx[i * NX + j];
        for (int i = 0; i < NX; ++i) sq->q[i] = gx[i];
        if (mode_lsq) {
            for (int i = 0; i < NX; ++i) sq->Q[i * NA + i] = 1.0;
            for (int j = 0; j < 3; ++j)
                sq->q[10 + j] += -W->zLw[k * 3 + j] + W->zUw[k * 3 + j];
        } else {
            for (int i = 0; i < NX; ++i) sq->Q[i * NA + i] += delta_w;
            for (int j = 0; j < 3; ++j) {
                double gb, sg;
                bar_terms(xk[10 + j], W->wlo, W->whi, W->zLw[k * 3 + j], W->zUw[k * 3 + j], W->mu, &gb, &sg);
                sq->Q[(10 + j) * NA + 10 + j] += sg;
                sq->q[10 + j] += gb;
            }
        }
        for (int i = 0; i < NX; ++i)
            for (int j = 0; j < NU; ++j) sq->S[i * NU + j] = Hxu[i * NU + j];
    }
    /* u_prev block (only k>=1 carries a free u_{k-1}) */
    const double *up = (k == 0) ? I->ulast : W->u + (k - 1) * NU;
    for (int j = 0; j < NU; ++j) {
        if (!mode_lsq) {
            sq->Q[(NX + j) * NA + NX + j] = 2 * P->du_weight * s;
            sq->S[(NX + j) * NU + j] = -2 * P->du_weight * s;
        }
        sq->q[NX + j] = -2 * P->du_weight * s * (uk[j] - up[j]);
    }
    /* u block */
    for (int j = 0; j < NU; ++j) {
        sq->r[j] = s * (2 * P->wthrust * uk[j] + 2 * P->du_weight * (uk[j] - up[j]));
        if (mode_lsq) {
            sq->R[j * NU + j] = 1.0;
            sq->r[j] += -W->zLu[k * NU + j] + W->zUu[k * NU + j];
        } else {
            double gb, sg;
            bar_terms(uk[j], W->ulo, W->uhi, W->zLu[k * NU + j], W->zUu[k * NU + j], W->mu, &gb, &sg);
            sq->R[j * NU + j] = s * (2 * P->wthrust + 2 * P->du_weight) + sg + delta_w;
            sq->r[j] += gb;
        }
    }
    if (W->refine) {
        for (int i = 0; i < NX; ++i) sq->q[i] = (k >= 1) ? W->rq[k * NX + i] : 0.0;
        for (int j = 0; j < NU; ++j) sq->q[NX + j] = 0.0;
        for (int j = 0; j < NU; ++j) sq->r[j] = W->rr[k * NU + j];
        for (int i = 0; i < NX; ++i) sq->c[i] = W->rc[k * NX + i];
    }
}

/* terminal value function (17x17, 17) */
static void build_terminal(const orc_params *P, const orc_inst *I, orc_ws *W, double delta_w, int mode_lsq,
                           double *Pm, double *p)
{
    memset(Pm, 0, sizeof(double) * NA * NA);
    memset(p, 0, sizeof(double) * NA);
    const int N = W->N;
    const double *xN = W->x + N * NX;
    double g[NX], H[NX * NX];
    memset(H, 0, sizeof(H));
    state_cost_derivs(P, &W->at, I->goal, I->ptra, 0.0, xN, g, H);
    for (int i = 0; i < NX; ++i) p[i] = W->s_obj * g[i];
    if (mode_lsq) {
        for (int i = 0; i < NX; ++i) Pm[i * NA + i] = 1.0;
        for (int j = 0; j < 3; ++j) p[10 + j] += -W->zLw[N * 3 + j] + W->zUw[N * 3 + j];
        return;
    }
    for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NX; ++j) Pm[i * NA + j] = W->s_obj * H[i * NX + j];
    for (int i = 0; i < NX; ++i) Pm[i * NA + i] += delta_w;
    for (int j = 0; j < 3; ++j) {
        double gb, sg;
        bar_terms(xN[10 + j], W->wlo, W->whi, W->zLw[N * 3 + j], W->zUw[N * 3 + j], W->mu, &gb, &sg);
        Pm[(10 + j) * NA + 10 + j] += sg;
        p[10 + j] += gb;
    }
    if (W->refine) {
        for (int i = 0; i < NX; ++i) p[i] = W->rq[N * NX + i];
        for (int j = 0; j < NU; ++j) p[NX + j] = 0.0;
    }
}

/* Riccati backward + forward + adjoint.  Returns 0 ok, -1 inertia (some Quu not PD). */
static int riccati_solve(const orc_params *P, const orc_inst *I, orc_ws *W, double delta_w, int mode_lsq)
{
    const int N = W->N;
    double Pm[NA * NA], p[NA];
    build_terminal(P, I, W, delta_w, mode_lsq, Pm, p);
    stage_qp sq;
    for (int k = N - 1; k >= 0; --k) {
        build_stage(P, I, W, k, delta_w, mode_lsq, &sq);
        /* PA = P * A~  (17x13 meaningful), PB = P * B~ (17x4) */
        double PA[NA * NX], PB[NA * NU], ph[NA];
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NX; ++j) {
                double acc = 0;
                for (int m = 0; m < NX; ++m) acc += Pm[i * NA + m] * sq.A[m * NX + j];
                PA[i * NX + j] = acc;
            }
            for (int j = 0; j < NU; ++j) {
                double acc = 0;
                for (int m = 0; m < NX; ++m) acc += Pm[i * NA + m] * sq.B[m * NU + j];
                acc += Pm[i * NA + NX + j];
                PB[i * NU + j] = acc;
            }
            double acc = p[i];
            for (int m = 0; m < NX; ++m) acc += Pm[i * NA + m] * sq.c[m];
            ph[i] = acc;
        }
        /* Quu = R + B~^T P B~ */
        double Quu[NU * NU], Qux[NU * NA], qu[NU];
        for (int a = 0; a < NU; ++a) {
            for (int b = 0; b < NU; ++b) {
                double acc = sq.R[a * NU + b];
                for (int m = 0; m < NX; ++m) acc += sq.B[m * NU + a] * PB[m * NU + b];
                acc += PB[(NX + a) * NU + b];
                Quu[a * NU + b] = acc;
            }
            /* Qux = S^T + B~^T P A~ : columns 0..12 from PA, columns 13..16 zero (A~ has zero u-cols) */
            for (int j = 0; j < NA; ++j) {
                double acc = sq.S[j * NU + a];
                if (j < NX) {
                    for (int m = 0; m < NX; ++m) acc += sq.B[m * NU + a] * PA[m * NX + j];
                    acc += PA[(NX + a) * NX + j];
                }
                Qux[a * NA + j] = acc;
            }
            double acc = sq.r[a];
            for (int m = 0; m < NX; ++m) acc += sq.B[m * NU + a] * ph[m];
            acc += ph[NX + a];
            qu[a] = acc;
        }
        /* symmetrize Quu */
        for (int a = 0; a < NU; ++a)
            for (int b = a + 1; b < NU; ++b) {
                double v = 0.5 * (Quu[a * NU + b] + Quu[b * NU + a]);
                Quu[a * NU + b] = Quu[b * NU + a] = v;
            }
        double L[20];
        if (chol4(Quu, L) != 0) {
#ifdef ORC_TRACE
            fprintf(stderr, "   chol fail k=%d dw=%.2e Quu diag %.3e %.3e %.3e %.3e  Pdiag(w) %.3e %.3e %.3e\n", k, delta_w,
                    Quu[0], Quu[5], Quu[10], Quu[15], Pm[10*NA+10], Pm[11*NA+11], Pm[12*NA+12]);
#endif
            return -1;
        }
        double *K = W->K + k * NU * NA, *kk = W->kff + k * NU;
        for (int j = 0; j < NA; ++j) {
            double col[NU];
            for (int a = 0; a < NU; ++a) col[a] = Qux[a * NA + j];
            chol4_solve(L, col);
            for (int a = 0; a < NU; ++a) K[a * NA + j] = -col[a];
        }
        {
            double col[NU];
            for (int a = 0; a < NU; ++a) col[a] = qu[a];
            chol4_solve(L, col);
            for (int a = 0; a < NU; ++a) kk[a] = -col[a];
        }
        if (k == 0) break;
        /* Qxx = Q + A~^T P A~ ; qx = q + A~^T ph ; Pnew = Qxx + Qux^T K ; pnew = qx + Qux^T k */
        double Pn[NA * NA], pn[NA];
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NA; ++j) {
                double acc = sq.Q[i * NA + j];
                if (i < NX && j < NX)
                    for (int m = 0; m < NX; ++m) acc += sq.A[m * NX + i] * PA[m * NX + j];
                for (int a = 0; a < NU; ++a) acc += Qux[a * NA + i] * K[a * NA + j];
                Pn[i * NA + j] = acc;
            }
            double acc = sq.q[i];
            if (i < NX)
                for (int m = 0; m < NX; ++m) acc += sq.A[m * NX + i] * ph[m];
            for (int a = 0; a < NU; ++a) acc += Qux[a * NA + i] * kk[a];
            pn[i] = acc;
        }
        for (int i = 0; i < NA; ++i)
            for (int j = 0; j < NA; ++j) Pm[i * NA + j] = 0.5 * (Pn[i * NA + j] + Pn[j * NA + i]);
        memcpy(p, pn, sizeof(pn));
    }
    /* forward */
    double dxa[NA];
    memset(dxa, 0, sizeof(dxa));
    memset(W->dx, 0, sizeof(double) * NX);
    for (int k = 0; k < N; ++k) {
        build_stage(P, I, W, k, delta_w, mode_lsq, &sq);
        const double *K = W->K + k * NU * NA, *kk = W->kff + k * NU;
        double duk[NU];
        for (int a = 0; a < NU; ++a) {
            double acc = kk[a];
            for (int j = 0; j < NA; ++j) acc += K[a * NA + j] * dxa[j];
            duk[a] = acc;
            W->du[k * NU + a] = acc;
        }
        double nx[NA];
        for (int i = 0; i < NX; ++i) {
            double acc = sq.c[i];
            for (int m = 0; m < NX; ++m) acc += sq.A[i * NX + m] * dxa[m];
            for (int a = 0; a < NU; ++a) acc += sq.B[i * NU + a] * duk[a];
            nx[i] = acc;
        }
        for (int a = 0; a < NU; ++a) nx[NX + a] = duk[a];
        memcpy(dxa, nx, sizeof(nx));
        memcpy(W->dx + (k + 1) * NX, nx, sizeof(double) * NX);
    }
    /* adjoint: lam+_{N-1} = Q_N dx_N + q_N ; lam+_{k-1} = Qxx_k dx_k + Sxu_k du_k + q_k + A_k^T lam+_k */
    {
        double PmN[NA * NA], pN[NA];
        build_terminal(P, I, W, delta_w, mode_lsq, PmN, pN);
        double *lp = W->lamp + (N - 1) * NX;
        for (int i = 0; i < NX; ++i) {
            double acc = pN[i];
            for (int j = 0; j < NX; ++j) acc += PmN[i * NA + j] * W->dx[N * NX + j];
            lp[i] = acc;
        }
        for (int k = N - 1; k >= 1; --k) {
            build_stage(P, I, W, k, delta_w, mode_lsq, &sq);
            const double *dxk = W->dx + k * NX, *duk = W->du + k * NU, *ln = W->lamp + k * NX;
            double *lo = W->lamp + (k - 1) * NX;
            for (int i = 0; i < NX; ++i) {
                double acc = sq.q[i];
                for (int j = 0; j < NX; ++j) acc += sq.Q[i * NA + j] * dxk[j];
                for (int a = 0; a < NU; ++a) acc += sq.S[i * NU + a] * duk[a];
                for (int m = 0; m < NX; ++m) acc += sq.A[m * NX + i] * ln[m];
                lo[i] = acc;
            }
        }
    }
    return 0;
}

/* Residual of the full (unreduced) primal-dual Newton system at the computed step (dx, du, lamp):
 *   rho_u,k = H_uu du_k + H_ux dx_k + H_{u_k u_k+-1} du_k+-1 + grad phi_u,k + B_k^T lam+_k
 *   rho_c,k = A_k dx_k + B_k du_k + c_k - dx_{k+1}
 *   rho_x,k = (H_xx + Sigma + dw) dx_k + H_xu du_k + grad phi_x,k - lam+_{k-1} + A_k^T lam+_k
 * Returns ||rho||_inf / (min(||sol||, 1e6 ||rhs||) + ||rhs||)  (IPOPT's residual ratio). */
static double kkt_residual(const orc_params *P, const orc_inst *I, orc_ws *W, double delta_w)
{
    const int N = W->N;
    const double s = W->s_obj;
    stage_qp sq;
    double nres = 0, nsol = 0, nrhs = 0;
    W->refine = 0;
    for (int k = 0; k < N; ++k) {
        build_stage(P, I, W, k, delta_w, 0, &sq);
        const double *dxk = W->dx + k * NX, *duk = W->du + k * NU, *lk = W->lamp + k * NX;
        /* u rows: R (which holds 2s for stage k's own smoothing) + 2s from stage k+1's smoothing */
        for (int a = 0; a < NU; ++a) {
            double acc = sq.R[a * NU + a] * duk[a];
            if (k + 1 < N) acc += 2 * P->du_weight * s * (duk[a] - W->du[(k + 1) * NU + a]);
            if (k >= 1) acc += -2 * P->du_weight * s * W->du[(k - 1) * NU + a];
            if (k >= 1)
                for (int i = 0; i < NX; ++i) acc += sq.S[i * NU + a] * dxk[i];
            double g = sq.r[a];
            /* full gradient of phi w.r.t. u_k includes stage k+1's smoothing term */
            if (k + 1 < N) g += -2 * P->du_weight * s * (W->u[(k + 1) * NU + a] - W->u[k * NU + a]);
            acc += g;
            for (int i = 0; i < NX; ++i) acc += sq.B[i * NU + a] * lk[i];
            W->rr[k * NU + a] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(g));
            nsol = fmax(nsol, fabs(duk[a]));
        }
        for (int i = 0; i < NX; ++i) {
            double acc = sq.c[i] - W->dx[(k + 1) * NX + i];
            for (int m = 0; m < NX; ++m) acc += sq.A[i * NX + m] * dxk[m];
            for (int a = 0; a < NU; ++a) acc += sq.B[i * NU + a] * duk[a];
            W->rc[k * NX + i] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(sq.c[i]));
            nsol = fmax(nsol, fabs(lk[i]));
        }
        if (k >= 1) {
            for (int i = 0; i < NX; ++i) {
                double acc = sq.q[i] - W->lamp[(k - 1) * NX + i];
                for (int j = 0; j < NX; ++j) acc += sq.Q[i * NA + j] * dxk[j];
                for (int a = 0; a < NU; ++a) acc += sq.S[i * NU + a] * duk[a];
                for (int m = 0; m < NX; ++m) acc += sq.A[m * NX + i] * lk[m];
                W->rq[k * NX + i] = acc;
                nres = fmax(nres, fabs(acc));
                nrhs = fmax(nrhs, fabs(sq.q[i]));
                nsol = fmax(nsol, fabs(dxk[i]));
            }
        }
    }
    {
        double Pm[NA * NA], p[NA];
        build_terminal(P, I, W, delta_w, 0, Pm, p);
        const double *dxN = W->dx + N * NX;
        for (int i = 0; i < NX; ++i) {
            double acc = p[i] - W->lamp[(N - 1) * NX + i];
            for (int j = 0; j < NX; ++j) acc += Pm[i * NA + j] * dxN[j];
            W->rq[N * NX + i] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(p[i]));
            nsol = fmax(nsol, fabs(dxN[i]));
        }
    }
    if (nrhs + nres == 0.0) return nres;
    return nres / (fmin(nsol, 1e6 * nrhs) + nrhs);
}

static int riccati_solve(const orc_params *P, const orc_inst *I, orc_ws *W, double delta_w, int mode_lsq);

/* Solve the Newton system with IPOPT-style iterative refinement (min 1, max 10 steps, stop at
 * residual ratio <= 1e-10 or when the ratio stops improving).  Returns 0 ok, -1 inertia. */
static void dump_step(const orc_ws *W, double *out)
{
    memcpy(out, W->dx, sizeof(double) * (W->N + 1) * NX);
    memcpy(out + (NMAX_DUMP + 1) * NX, W->du, sizeof(double) * W->N * NU);
    memcpy(out + (NMAX_DUMP + 1) * NX + NMAX_DUMP * NU, W->lamp, sizeof(double) * W->N * NX);
}

/* IPOPT's iterative refinement of a computed solution (min 1, max 10 steps; stop at residual ratio
 * <= 1e-10 or when the ratio stops improving), starting from residual ratio `ratio` */
static void refine_loop(const orc_params *P, const orc_inst *I, orc_ws *W, double delta_w, double ratio, double *ratios)
{
    double dx[(NMAX + 1) * NX], du[NMAX * NU], dl[NMAX * NX];
    for (int step = 0; step < 10; ++step) {
        if (step >= 1 && ratio <= 1e-10) break;
        memcpy(dx, W->dx, sizeof(double) * (W->N + 1) * NX);
        memcpy(du, W->du, sizeof(double) * W->N * NU);
        memcpy(dl, W->lamp, sizeof(double) * W->N * NX);
        W->refine = 1;
        riccati_solve(P, I, W, delta_w, 0);   /* same matrices: inertia already known */
        W->refine = 0;
        W->sweeps++;
        W->refines++;
        /* the refinement sweep returned D = -K^{-1} rho: sol <- sol + D */
        for (int i = 0; i < (W->N + 1) * NX; ++i) W->dx[i] = dx[i] + W->dx[i];
        for (int i = 0; i < W->N * NU; ++i) W->du[i] = du[i] + W->du[i];
        for (int i = 0; i < W->N * NX; ++i) W->lamp[i] = dl[i] + W->lamp[i];
        double nr = kkt_residual(P, I, W, delta_w);
        if (step < 2) ratios[1 + step] = nr;
        ratios[3] += 1;
        if (!(nr < ratio)) {   /* no improvement: undo this correction and stop */
            memcpy(W->dx, dx, sizeof(double) * (W->N + 1) * NX);
            memcpy(W->du, du, sizeof(double) * W->N * NU);
            memcpy(W->lamp, dl, sizeof(double) * W->N * NX);
            break;
        }
        ratio = nr;
    }
}

static int newton_step(const orc_params *P, const orc_inst *I, orc_ws *W, double delta_w, double *ratios,
                       double *dump_pre)
{
    W->refine = 0;
    int rc = riccati_solve(P, I, W, delta_w, 0);
    W->sweeps++;
    if (rc != 0) return rc;
    if (dump_pre) dump_step(W, dump_pre);
    double ratio = kkt_residual(P, I, W, delta_w);
    ratios[0] = ratio; ratios[1] = -1; ratios[2] = -1; ratios[3] = 0;
    refine_loop(P, I, W, delta_w, ratio, ratios);
    return 0;
}

/* c[k] = f_d(x_k, u_k) - x_{k+1} at x + alpha dx, u + alpha du (the trial point of eval_merit) */
static void trial_defects(const orc_params *P, orc_ws *W, double alpha, double *c)
{
    for (int k = 0; k < W->N; ++k) {
        double xk[NX], uk[NU], xn[NX];
        for (int i = 0; i < NX; ++i) xk[i] = W->x[k * NX + i] + alpha * W->dx[k * NX + i];
        for (int j = 0; j < NU; ++j) uk[j] = W->u[k * NU + j] + alpha * W->du[k * NU + j];
        f_disc(P, xk, uk, xn);
        for (int i = 0; i < NX; ++i) c[k * NX + i] = xn[i] - (W->x[(k + 1) * NX + i] + alpha * W->dx[(k + 1) * NX + i]);
    }
}

/* Second-order-correction direction (IPOPT FilterLSAcceptor::TrySecondOrderCorrection): the Newton system of
 * this iteration (same matrix, same delta_w, no new factorisation) with the constraint part replaced by
 * c_soc = W->cs.  Solved as one sweep with right-hand side (grad phi, c_soc) through the refinement
 * path, then refined like any step. */
static void soc_direction(const orc_params *P, const orc_inst *I, orc_ws *W, double delta_w, double *ratios)
{
    const int N = W->N;
    for (int k = 0; k < N; ++k) {
        double g[NX], gu[NU];
        grad_u(P, I, W, k, gu);
        for (int j = 0; j < NU; ++j) {
            double gb, sg;
            bar_terms(W->u[k * NU + j], W->ulo, W->uhi, 0, 0, W->mu, &gb, &sg);
            W->rr[k * NU + j] = gu[j] + gb;
        }
        const int k1 = k + 1;
        grad_x(P, I, W, k1, g);
        for (int c = 0; c < 3; ++c) {
            double gb, sg;
            bar_terms(W->x[k1 * NX + 10 + c], W->wlo, W->whi, 0, 0, W->mu, &gb, &sg);
            g[10 + c] += gb;
        }
        for (int i = 0; i < NX; ++i) W->rq[k1 * NX + i] = g[i];
        for (int i = 0; i < NX; ++i) W->rc[k * NX + i] = W->cs[k * NX + i];
    }
    W->refine = 1;
    riccati_solve(P, I, W, delta_w, 0);
    W->refine = 0;
    W->sweeps++;
    W->soc = 1;
    double ratio = kkt_residual(P, I, W, delta_w);
    refine_loop(P, I, W, delta_w, ratio, ratios);
    W->soc = 0;
}

/* ---- optimality errors ------------------------------------------------------------------ */
typedef struct {
    double dual_inf, primal_inf, compl_mu, compl_0, s_d, s_c;
    double dual_inf_unscaled;
    int arg_type, arg_k, arg_i;
} kkt_err;

static void compute_errors(const orc_params *P, const orc_inst *I, orc_ws *W, double mu, kkt_err *E)
{
    const int N = W->N;
    double dinf = 0, pinf = 0, cmu = 0, c0 = 0, sum_mult = 0, sum_z = 0;
    double A[NX * NX], B[NX * NU];
    /* u gradients */
    for (int k = 0; k < N; ++k) {
        double g[NU];
        grad_u(P, I, W, k, g);
        jac_disc(P, W->x + k * NX, W->u + k * NU, A, B);
        const double *lk = W->lam + k * NX;
        for (int j = 0; j < NU; ++j) {
            double acc = g[j];
            for (int i = 0; i < NX; ++i) acc += B[i * NU + j] * lk[i];
            acc += -W->zLu[k * NU + j] + W->zUu[k * NU + j];
            if (fabs(acc) > dinf) {
                dinf = fabs(acc);
#ifdef ORC_TRACE
                E->arg_type = 0; E->arg_k = k; E->arg_i = j;
#endif
            }
            double v = W->u[k * NU + j];
            double sl = v - W->ulo, su = W->uhi - v;
            double zl = W->zLu[k * NU + j], zu = W->zUu[k * NU + j];
            cmu = fmax(cmu, fmax(fabs(sl * zl - mu), fabs(su * zu - mu)));
            c0 = fmax(c0, fmax(fabs(sl * zl), fabs(su * zu)));
            sum_z += zl + zu;
        }
        double xn[NX];
        f_disc(P, W->x + k * NX, W->u + k * NU, xn);
        for (int i = 0; i < NX; ++i) {
            double d = fabs(xn[i] - W->x[(k + 1) * NX + i]);
            if (d > pinf) pinf = d;
            sum_mult += fabs(lk[i]);
        }
    }
    /* x gradients (k = 1..N) */
    for (int k = 1; k <= N; ++k) {
        double g[NX];
        grad_x(P, I, W, k, g);
        for (int i = 0; i < NX; ++i) g[i] -= W->lam[(k - 1) * NX + i];
        if (k < N) {
            jac_disc(P, W->x + k * NX, W->u + k * NU, A, B);
            const double *lk = W->lam + k * NX;
            for (int i = 0; i < NX; ++i)
                for (int m = 0; m < NX; ++m) g[i] += A[m * NX + i] * lk[m];
        }
        for (int j = 0; j < 3; ++j) {
            g[10 + j] += -W->zLw[k * 3 + j] + W->zUw[k * 3 + j];
            double v = W->x[k * NX + 10 + j];
            double sl = v - W->wlo, su = W->whi - v;
            double zl = W->zLw[k * 3 + j], zu = W->zUw[k * 3 + j];
            cmu = fmax(cmu, fmax(fabs(sl * zl - mu), fabs(su * zu - mu)));
            c0 = fmax(c0, fmax(fabs(sl * zl), fabs(su * zu)));
            sum_z += zl + zu;
        }
        for (int i = 0; i < NX; ++i)
            if (fabs(g[i]) > dinf) {
                dinf = fabs(g[i]);
#ifdef ORC_TRACE
                E->arg_type = 1; E->arg_k = k; E->arg_i = i;
#endif
            }
    }
    const double s_max = 100.0;
    double n_mult = (double)(N * NX) + (double)(N * NU * 2 + N * 3 * 2);
    double n_z = (double)(N * NU * 2 + N * 3 * 2);
    E->s_d = fmax(s_max, (sum_mult + sum_z) / n_mult) / s_max;
    E->s_c = fmax(s_max, sum_z / n_z) / s_max;
    E->dual_inf = dinf;
    E->primal_inf = pinf;
    E->compl_mu = cmu;
    E->compl_0 = c0;
    E->dual_inf_unscaled = dinf / W->s_obj;
}

/* mu^1.5 of IPOPT's monotone barrier update (mu_new = max(mu_min, min(kappa_mu mu, mu^theta_mu)), theta_mu = 1.5),
 * correctly rounded: sqrt and the product in double-double, rounded once (libm pow is within about half an ulp; the
 * device uses this same function, ipm_kernel.hip pow15, so that both take the same mu sequence bit for bit) */
static double pow15(double x)
{
    const double s = sqrt(x);
    const double slo = fma(-s, s, x) / (2.0 * s);
    const double p = x * s;
    const double plo = fma(x, s, -p);
    return p + fma(x, slo, plo);
}

static double err_value(const kkt_err *E, int with_mu)
{
    double c = with_mu ? E->compl_mu : E->compl_0;
    return fmax(E->dual_inf / E->s_d, fmax(E->primal_inf, c / E->s_c));
}

/* ---- line search pieces ----------------------------------------------------------------- */
/* primal fraction-to-the-boundary step of (du, dx) (bounded components: u, omega) */
static double primal_ftb(const orc_ws *W, double tau)
{
    const int N = W->N;
    double amax = 1.0;
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < NU; ++j) {
            double v = W->u[k * NU + j], d = W->du[k * NU + j];
            double sl = v - W->ulo, su = W->uhi - v;
            if (d < 0) amax = fmin(amax, -tau * sl / d);
            if (d > 0) amax = fmin(amax, tau * su / d);
        }
    for (int k = 1; k <= N; ++k)
        for (int j = 0; j < 3; ++j) {
            double v = W->x[k * NX + 10 + j], d = W->dx[k * NX + 10 + j];
            double sl = v - W->wlo, su = W->whi - v;
            if (d < 0) amax = fmin(amax, -tau * sl / d);
            if (d > 0) amax = fmin(amax, tau * su / d);
        }
    return amax;
}

/* dual fraction-to-the-boundary step of the bound multipliers implied by (du, dx) */
static double dual_ftb(const orc_ws *W, double tau, double mu)
{
    const int N = W->N;
    double az = 1.0;
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < NU; ++j) {
            double v = W->u[k * NU + j], d = W->du[k * NU + j];
            double sl = v - W->ulo, su = W->uhi - v;
            double zl = W->zLu[k * NU + j], zu = W->zUu[k * NU + j];
            double dzl = mu / sl - zl - zl / sl * d;
            double dzu = mu / su - zu + zu / su * d;
            if (dzl < 0) az = fmin(az, -tau * zl / dzl);
            if (dzu < 0) az = fmin(az, -tau * zu / dzu);
        }
    for (int k = 1; k <= N; ++k)
        for (int j = 0; j < 3; ++j) {
            double v = W->x[k * NX + 10 + j], d = W->dx[k * NX + 10 + j];
            double sl = v - W->wlo, su = W->whi - v;
            double zl = W->zLw[k * 3 + j], zu = W->zUw[k * 3 + j];
            double dzl = mu / sl - zl - zl / sl * d;
            double dzu = mu / su - zu + zu / su * d;
            if (dzl < 0) az = fmin(az, -tau * zl / dzl);
            if (dzu < 0) az = fmin(az, -tau * zu / dzu);
        }
    return az;
}

/* IPOPT FilterLSAcceptor::CheckAcceptabilityOfTrialPoint: switching condition / Armijo with the step
 * size alpha_test of the original direction, sufficient decrease otherwise, then the filter */
static int ls_accept(double alpha_test, double tht, double pht, int okt, double th0, double ph0, double gBD,
                     double theta_max, double theta_min, const double *filt_t, const double *filt_p, int nfilt)
{
    const double eps = 2.220446049250313e-16;
    int acc = okt && !(tht > theta_max);
    if (acc) {
        int ftype = (gBD < 0) && (alpha_test * pow(-gBD, 2.3) > pow(th0, 1.1));
        if (ftype && th0 <= theta_min) {
            acc = (pht - ph0 - 1e-8 * alpha_test * gBD) <= 10.0 * eps * fabs(ph0);
        } else {
            int objinc_ok = 1;
            if (pht > ph0) {
                double basval = (fabs(ph0) > 10.0) ? log10(fabs(ph0)) : 1.0;
                if (log10(pht - ph0) > 5.0 + basval) objinc_ok = 0;
            }
            acc = objinc_ok && (((tht - (1.0 - 1e-5) * th0) <= 10.0 * eps * fabs(th0)) ||
                                ((pht - ph0 + 1e-8 * th0) <= 10.0 * eps * fabs(ph0)));
        }
    }
    if (acc)
        for (int f = 0; f < nfilt; ++f)
            if (!(tht <= filt_t[f] || pht <= filt_p[f])) return 0;
    return acc;
}

static void trial_merit(const orc_params *P, const orc_inst *I, orc_ws *W, double alpha, double mu, double *tht,
                        double *pht, int *okt)
{
    double xt[(NMAX + 1) * NX], ut[NMAX * NU];
    for (int k = 0; k < (W->N + 1) * NX; ++k) xt[k] = W->x[k] + alpha * W->dx[k];
    for (int k = 0; k < W->N * NU; ++k) ut[k] = W->u[k] + alpha * W->du[k];
    eval_merit(P, I, W, xt, ut, mu, tht, pht, okt);
    W->trials++;
}

/* ---- soft restoration phase ----------------------------------------------------------------
 * IPOPT 3.12 BacktrackingLineSearch: when the backtracking line search fails, IPOPT first tries the "soft
 * restoration phase" before the restoration phase proper (options soft_resto_pderror_reduction_factor = 0.9999,
 * max_soft_resto_iters = 10): the full fraction-to-the-boundary step alpha = min(alpha_primal_max, alpha_dual_max)
 * of the current search direction for the primal variables and all multipliers is accepted when it reduces the
 * primal-dual system error by that factor (TrySoftRestoStep); when the trial point is also acceptable to the
 * original filter line search (CheckAcceptabilityOfTrialPoint(0)) the soft phase ends, otherwise the next
 * iterations continue with such steps, for at most max_soft_resto_iters of them. */

/* IpoptCalculatedQuantities::*_primal_dual_system_error(mu): l1 norms of the (scaled) dual infeasibility, the
 * primal infeasibility and the mu-complementarity.  IPOPT divides the sum by the number of its terms; the soft
 * restoration test compares two such values of the same problem, where the common divisor drops out. */
static double pd_system_error(const orc_params *P, const orc_inst *I, orc_ws *W, double mu)
{
    const int N = W->N;
    double dual = 0, primal = 0, cmpl = 0;
    double A[NX * NX], B[NX * NU];
    for (int k = 0; k < N; ++k) {
        double g[NU];
        grad_u(P, I, W, k, g);
        jac_disc(P, W->x + k * NX, W->u + k * NU, A, B);
        const double *lk = W->lam + k * NX;
        for (int j = 0; j < NU; ++j) {
            double acc = g[j];
            for (int i = 0; i < NX; ++i) acc += B[i * NU + j] * lk[i];
            acc += -W->zLu[k * NU + j] + W->zUu[k * NU + j];
            dual += fabs(acc);
            const double v = W->u[k * NU + j];
            cmpl += fabs((v - W->ulo) * W->zLu[k * NU + j] - mu) + fabs((W->uhi - v) * W->zUu[k * NU + j] - mu);
        }
        double xn[NX];
        f_disc(P, W->x + k * NX, W->u + k * NU, xn);
        for (int i = 0; i < NX; ++i) primal += fabs(xn[i] - W->x[(k + 1) * NX + i]);
    }
    for (int k = 1; k <= N; ++k) {
        double g[NX];
        grad_x(P, I, W, k, g);
        for (int i = 0; i < NX; ++i) g[i] -= W->lam[(k - 1) * NX + i];
        if (k < N) {
            jac_disc(P, W->x + k * NX, W->u + k * NU, A, B);
            const double *lk = W->lam + k * NX;
            for (int i = 0; i < NX; ++i)
                for (int m = 0; m < NX; ++m) g[i] += A[m * NX + i] * lk[m];
        }
        for (int j = 0; j < 3; ++j) {
            g[10 + j] += -W->zLw[k * 3 + j] + W->zUw[k * 3 + j];
            const double v = W->x[k * NX + 10 + j];
            cmpl += fabs((v - W->wlo) * W->zLw[k * 3 + j] - mu) + fabs((W->whi - v) * W->zUw[k * 3 + j] - mu);
        }
        for (int i = 0; i < NX; ++i) dual += fabs(g[i]);
    }
    return dual + primal + cmpl;
}

/* the iterate after a step: primal and constraint multipliers with alpha, bound multipliers with alpha_z (their
 * steps from the old slacks), then IPOPT's kappa_sigma safeguard (AcceptTrialPoint) when `safeguard` */
static void take_step(orc_ws *W, double alpha, double az, double mu, int safeguard)
{
    const int N = W->N;
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < NU; ++j) {
            double v = W->u[k * NU + j], d = W->du[k * NU + j];
            double sl = v - W->ulo, su = W->uhi - v;
            double zl = W->zLu[k * NU + j], zu = W->zUu[k * NU + j];
            double dzl = mu / sl - zl - zl / sl * d;
            double dzu = mu / su - zu + zu / su * d;
            W->zLu[k * NU + j] = zl + az * dzl;
            W->zUu[k * NU + j] = zu + az * dzu;
        }
    for (int k = 1; k <= N; ++k)
        for (int j = 0; j < 3; ++j) {
            double v = W->x[k * NX + 10 + j], d = W->dx[k * NX + 10 + j];
            double sl = v - W->wlo, su = W->whi - v;
            double zl = W->zLw[k * 3 + j], zu = W->zUw[k * 3 + j];
            double dzl = mu / sl - zl - zl / sl * d;
            double dzu = mu / su - zu + zu / su * d;
            W->zLw[k * 3 + j] = zl + az * dzl;
            W->zUw[k * 3 + j] = zu + az * dzu;
        }
    for (int k = 0; k < N * NX; ++k) W->lam[k] += alpha * (W->lamp[k] - W->lam[k]);
    for (int k = 0; k < (N + 1) * NX; ++k) W->x[k] += alpha * W->dx[k];
    for (int k = 0; k < N * NU; ++k) W->u[k] += alpha * W->du[k];
    if (!safeguard) return;
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < NU; ++j) {
            double v = W->u[k * NU + j];
            double sl = v - W->ulo, su = W->uhi - v;
            double *zl = &W->zLu[k * NU + j], *zu = &W->zUu[k * NU + j];
            *zl = fmax(fmin(*zl, 1e10 * mu / sl), mu / (1e10 * sl));
            *zu = fmax(fmin(*zu, 1e10 * mu / su), mu / (1e10 * su));
        }
    for (int k = 1; k <= N; ++k)
        for (int j = 0; j < 3; ++j) {
            double v = W->x[k * NX + 10 + j];
            double sl = v - W->wlo, su = W->whi - v;
            double *zl = &W->zLw[k * 3 + j], *zu = &W->zUw[k * 3 + j];
            *zl = fmax(fmin(*zl, 1e10 * mu / sl), mu / (1e10 * sl));
            *zu = fmax(fmin(*zu, 1e10 * mu / su), mu / (1e10 * su));
        }
}

/* TrySoftRestoStep: returns 1 when the step alpha_s = min(amax, az) reduces the primal-dual system error by
 * 0.9999 (*alpha_s set; *orig: the trial point also passes the original filter line-search test with
 * alpha_test = 0, *tht / *pht its merit) */
static int try_soft_resto(const orc_params *P, const orc_inst *I, orc_ws *W, double mu, double amax, double az,
                          double th0, double ph0, double gBD, double theta_max, double theta_min, const double *filt_t,
                          const double *filt_p, int nfilt, double *alpha_s, int *orig, double *tht, double *pht)
{
    const double a = fmin(amax, az);
    const double cur = pd_system_error(P, I, W, mu);
    orc_ws *T = (orc_ws *)malloc(sizeof(orc_ws));
    memcpy(T, W, sizeof(orc_ws));
    take_step(T, a, a, mu, 0);
    const double trial = pd_system_error(P, I, T, mu);
    int okt = 1;
    eval_merit(P, I, T, T->x, T->u, mu, tht, pht, &okt);
    free(T);
    W->trials++;
    *alpha_s = a;
    *orig = 0;
    if (!(trial <= 0.9999 * cur)) return 0;
    *orig = ls_accept(0.0, *tht, *pht, okt, th0, ph0, gBD, theta_max, theta_min, filt_t, filt_p, nfilt);
    return 1;
}

/* ========================================================================================== */
/* Restoration phase (IPOPT 3.12 MinC_1NrmRestorationPhase on RestoIpoptNLP)                    */
/* ========================================================================================== */
/* Entered when the filter line search and the soft restoration phase both fail at a point that is not almost
 * feasible (theta > 1e-2 tol).  The restoration NLP, over the original free variables v = (x_1..x_N, u_0..u_{N-1})
 * and two slacks p, n >= 0 per equality constraint (N x 13 each):
 *     min  rho sum(p + n) + eta/2 ||D_R (v - v_R)||^2      s.t.  f_d(x_k, u_k) - x_{k+1} - p_k + n_k = 0,
 *          original bounds on v (u box, omega box, relaxed as in the original), p, n >= 0,
 * rho = resto_penalty_parameter = 1000, eta = sqrt(mu_R) (eta_factor 1, eta_mu_exponent 0.5, mu_R the current
 * restoration barrier parameter), v_R the point where the restoration starts, D_R = min(1, 1/|v_R|) elementwise.
 * It is solved by the same interior-point algorithm (barrier, monotone mu, inertia correction, iterative
 * refinement, filter line search with its own filter) and left as soon as an iterate is acceptable to the
 * original problem (RestoFilterConvergenceCheck): theta_orig <= 0.9 theta_R (required_infeasibility_reduction),
 * acceptable to the original filter, which was augmented with the start point, and sufficient decrease
 * against the start point.  Then the original iteration continues from v with the restoration's bound
 * multipliers (all reset to 1 when one exceeds bound_mult_reset_threshold = 1000) and zero constraint
 * multipliers (constr_mult_reset_threshold = 0).
 *
 * Newton system: after eliminating dp = (lam+ - r_p) / Sp and dn = (-lam+ - r_n) / Sn (Sp = z_p / p + delta_w,
 * r_p = rho - mu / p, likewise n), each constraint row becomes a soft dynamics equation
 *     dx_{k+1} = A dx_k + B du_k + c'_k - D_k lam+_k,   D = 1/Sp + 1/Sn,   c' = c_R + r_p / Sp - r_n / Sn,
 * and lam+_k = (P_{k+1} dx~_{k+1} + p_{k+1})_x.  The Riccati recursion then carries, ahead of every stage,
 * the value function through the infimal convolution with the soft constraint (see resto_transform); the
 * system has the correct inertia iff every I + D^1/2 P_xx D^1/2 and every Quu is positive definite.
 *
 * Assumptions where IPOPT's source is not at hand (documented in DESIGN.md): mu_R = max(mu, ||c||_inf), bound
 * multipliers of v start at min(rho, z), of p / n at mu_R / p, mu_R / n; constraint multipliers start at the
 * least-squares estimate when it is <= constr_mult_init_max (1000) in max norm, else 0; no second-order
 * corrections and no soft restoration inside the restoration phase; a failed restoration line search ends the
 * solve (IPOPT: Restoration_Failed).  Restoration iterations count as iterations. */
#define RESTO_RHO 1000.0
#define ST_RESTO_FAIL 8
#define ST_INFEASIBLE 9

typedef struct {
    double p[NMAX * NX], n[NMAX * NX], zp[NMAX * NX], zn[NMAX * NX];
    double dp[NMAX * NX], dn[NMAX * NX];
    double xR[(NMAX + 1) * NX], uR[NMAX * NU];    /* reference point */
    double dx2[(NMAX + 1) * NX], du2[NMAX * NU];  /* D_R^2 */
    double mu, eta;
    int refine;                                   /* 1: the p / n rows take their right-hand side from rp / rn */
    double rp[NMAX * NX], rn[NMAX * NX];
    /* per stage, kept by the backward sweep for the forward sweep: Cholesky of S' = I + D^1/2 P_xx D^1/2 of the
     * value function P_{k+1}, its sqrt(D), and P_{k+1}, p_{k+1} themselves */
    double Ls[NMAX][NX * NX], sD[NMAX][NX];
    double Pk1[NMAX][NA * NA], pk1[NMAX][NA];
    double Ks[NMAX * NU * NA], kff[NMAX * NU];
} resto_t;

static double eta_of(double mu) { return sqrt(mu); }

/* dense Cholesky of an n x n SPD matrix (row-major, lower L); returns -1 when a pivot is not positive */
static int cholN(int n, const double *M, double *L)
{
    memset(L, 0, sizeof(double) * n * n);
    for (int j = 0; j < n; ++j) {
        double d = M[j * n + j];
        for (int k = 0; k < j; ++k) d -= L[j * n + k] * L[j * n + k];
        if (!(d > 0.0)) return -1;
        const double ljj = sqrt(d);
        L[j * n + j] = ljj;
        for (int i = j + 1; i < n; ++i) {
            double s = M[i * n + j];
            for (int k = 0; k < j; ++k) s -= L[i * n + k] * L[j * n + k];
            L[i * n + j] = s / ljj;
        }
    }
    return 0;
}

/* L L^T x = b in place */
static void cholN_solve(int n, const double *L, double *b)
{
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * n + k] * b[k];
        b[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * b[k];
        b[i] = s / L[i * n + i];
    }
}

/* p / n row data of constraint row e: Sp', Sn' (with delta_w) and the linear terms r_p, r_n */
static void resto_pn_terms(const resto_t *R, int e, double delta_w, int mode_lsq, double *Sp, double *Sn, double *rp,
                           double *rn)
{
    if (mode_lsq) {
        *Sp = 1.0; *Sn = 1.0;
        *rp = RESTO_RHO - R->zp[e];
        *rn = RESTO_RHO - R->zn[e];
        return;
    }
    *Sp = R->zp[e] / R->p[e] + delta_w;
    *Sn = R->zn[e] / R->n[e] + delta_w;
    if (R->refine) {
        *rp = R->rp[e];
        *rn = R->rn[e];
    } else {
        *rp = RESTO_RHO - R->mu / R->p[e];
        *rn = RESTO_RHO - R->mu / R->n[e];
    }
}

/* stage QP of the restoration problem (layout of stage_qp: Q 17x17, S 17x4, R 4x4, q 17, r 4, A, B, c = c') */
static void build_stage_resto(const orc_params *P, orc_ws *W, const resto_t *R, int k, double delta_w, int mode_lsq,
                              stage_qp *sq, double *Dk)
{
    const double *xk = W->x + k * NX, *uk = W->u + k * NU;
    memset(sq, 0, sizeof(*sq));
    jac_disc(P, xk, uk, sq->A, sq->B);
    double xn[NX];
    f_disc(P, xk, uk, xn);
    const double eta = R->eta;
    if (k >= 1) {
        double Hxx[NX * NX], Hxu[NX * NU];
        memset(Hxx, 0, sizeof(Hxx));
        memset(Hxu, 0, sizeof(Hxu));
        if (!mode_lsq) hess_lam_disc(P, xk, uk, W->lam + k * NX, Hxx, Hxu);
        for (int i = 0; i < NX; ++i) {
            for (int j = 0; j < NX; ++j) sq->Q[i * NA + j] = Hxx[i * NX + j];
            for (int j = 0; j < NU; ++j) sq->S[i * NU + j] = Hxu[i * NU + j];
            sq->q[i] = eta * R->dx2[k * NX + i] * (xk[i] - R->xR[k * NX + i]);
            sq->Q[i * NA + i] += mode_lsq ? 1.0 : eta * R->dx2[k * NX + i] + delta_w;
        }
        for (int j = 0; j < 3; ++j) {
            if (mode_lsq) {
                sq->q[10 + j] += -W->zLw[k * 3 + j] + W->zUw[k * 3 + j];
            } else {
                double gb, sg;
                bar_terms(xk[10 + j], W->wlo, W->whi, W->zLw[k * 3 + j], W->zUw[k * 3 + j], R->mu, &gb, &sg);
                sq->Q[(10 + j) * NA + 10 + j] += sg;
                sq->q[10 + j] += gb;
            }
        }
    }
    for (int j = 0; j < NU; ++j) {
        sq->r[j] = eta * R->du2[k * NU + j] * (uk[j] - R->uR[k * NU + j]);
        if (mode_lsq) {
            sq->R[j * NU + j] = 1.0;
            sq->r[j] += -W->zLu[k * NU + j] + W->zUu[k * NU + j];
        } else {
            double gb, sg;
            bar_terms(uk[j], W->ulo, W->uhi, W->zLu[k * NU + j], W->zUu[k * NU + j], R->mu, &gb, &sg);
            sq->R[j * NU + j] = eta * R->du2[k * NU + j] + sg + delta_w;
            sq->r[j] += gb;
        }
    }
    if (W->refine) {
        for (int i = 0; i < NX; ++i) sq->q[i] = (k >= 1) ? W->rq[k * NX + i] : 0.0;
        for (int j = 0; j < NU; ++j) sq->r[j] = W->rr[k * NU + j];
    }
    for (int i = 0; i < NX; ++i) {
        const int e = k * NX + i;
        double Sp, Sn, rp, rn;
        resto_pn_terms(R, e, delta_w, mode_lsq, &Sp, &Sn, &rp, &rn);
        double c = 0.0;
        if (!mode_lsq) c = W->refine ? W->rc[e] : xn[i] - W->x[(k + 1) * NX + i] - R->p[e] + R->n[e];
        sq->c[i] = c + rp / Sp - rn / Sn;
        Dk[i] = 1.0 / Sp + 1.0 / Sn;
    }
}

static void build_terminal_resto(orc_ws *W, const resto_t *R, double delta_w, int mode_lsq, double *Pm, double *p)
{
    const int N = W->N;
    const double *xN = W->x + N * NX;
    memset(Pm, 0, sizeof(double) * NA * NA);
    memset(p, 0, sizeof(double) * NA);
    for (int i = 0; i < NX; ++i) {
        p[i] = R->eta * R->dx2[N * NX + i] * (xN[i] - R->xR[N * NX + i]);
        Pm[i * NA + i] = mode_lsq ? 1.0 : R->eta * R->dx2[N * NX + i] + delta_w;
    }
    for (int j = 0; j < 3; ++j) {
        if (mode_lsq) {
            p[10 + j] += -W->zLw[N * 3 + j] + W->zUw[N * 3 + j];
        } else {
            double gb, sg;
            bar_terms(xN[10 + j], W->wlo, W->whi, W->zLw[N * 3 + j], W->zUw[N * 3 + j], R->mu, &gb, &sg);
            Pm[(10 + j) * NA + 10 + j] += sg;
            p[10 + j] += gb;
        }
    }
    if (W->refine)
        for (int i = 0; i < NX; ++i) p[i] = W->rq[N * NX + i];
}

/* Value function (Pm, p) of x~_{k+1} -> the one of y' = G z + c' through the soft constraint with diagonal D
 * (x rows only; the u_prev rows are exact).  With s = sqrt(D), S' = I + diag(s) P_xx diag(s) = L L^T and
 * X = S'^-1 diag(s) [P_xx | P_xv | p_x]:  P^_xx = diag(1/s) X_xx (symmetrised), P^_xv = diag(1/s) X_xv,
 * P^_vv = P_vv - (diag(s) P_xv)^T X_xv, p^_x = diag(1/s) X_p, p^_v = p_v - (diag(s) P_xv)^T X_p.  Returns -1 when
 * S' is not positive definite (wrong inertia); L and s are kept for the forward sweep. */
static int resto_transform(double *Pm, double *p, const double *D, double *L, double *s)
{
    double Sm[NX * NX];
    for (int i = 0; i < NX; ++i) s[i] = sqrt(D[i]);
    for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NX; ++j) Sm[i * NX + j] = (i == j ? 1.0 : 0.0) + s[i] * Pm[i * NA + j] * s[j];
    if (cholN(NX, Sm, L) != 0) return -1;
    double X[NX][NA + 1];   /* columns 0..12: xx, 13..16: xv, 17: p */
    for (int c = 0; c < NA + 1; ++c) {
        double b[NX];
        for (int i = 0; i < NX; ++i) b[i] = s[i] * (c < NA ? Pm[i * NA + c] : p[i]);
        cholN_solve(NX, L, b);
        for (int i = 0; i < NX; ++i) X[i][c] = b[i];
    }
    double Pn[NA * NA], pn[NA];
    for (int i = 0; i < NX; ++i) {
        for (int j = 0; j < NA; ++j) Pn[i * NA + j] = X[i][j] / s[i];
        pn[i] = X[i][NA] / s[i];
    }
    for (int a = NX; a < NA; ++a) {
        for (int b = NX; b < NA; ++b) {
            double acc = Pm[a * NA + b];
            for (int i = 0; i < NX; ++i) acc -= s[i] * Pm[i * NA + a] * X[i][b];
            Pn[a * NA + b] = acc;
        }
        for (int j = 0; j < NX; ++j) Pn[a * NA + j] = Pn[j * NA + a];
        double acc = p[a];
        for (int i = 0; i < NX; ++i) acc -= s[i] * Pm[i * NA + a] * X[i][NA];
        pn[a] = acc;
    }
    for (int i = 0; i < NA; ++i)
        for (int j = 0; j < NA; ++j) Pm[i * NA + j] = 0.5 * (Pn[i * NA + j] + Pn[j * NA + i]);
    memcpy(p, pn, sizeof(pn));
    return 0;
}

/* Newton step of the restoration problem: Riccati with the soft-constraint transform; returns -1 on wrong inertia.
 * Fills W->dx, W->du, W->lamp (lam+), R->dp, R->dn. */
static int riccati_resto(const orc_params *P, orc_ws *W, resto_t *R, double delta_w, int mode_lsq)
{
    const int N = W->N;
    double Pm[NA * NA], p[NA];
    build_terminal_resto(W, R, delta_w, mode_lsq, Pm, p);
    stage_qp sq;
    double Dst[NMAX][NX], cst[NMAX][NX];
    for (int k = N - 1; k >= 0; --k) {
        build_stage_resto(P, W, R, k, delta_w, mode_lsq, &sq, Dst[k]);
        memcpy(cst[k], sq.c, sizeof(sq.c));
        memcpy(R->Pk1[k], Pm, sizeof(Pm));
        memcpy(R->pk1[k], p, sizeof(p));
        if (resto_transform(Pm, p, Dst[k], R->Ls[k], R->sD[k]) != 0) return -1;
        /* the stage with (Pm, p) = the transformed value function: as riccati_solve */
        double PA[NA * NX], PB[NA * NU], ph[NA];
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NX; ++j) {
                double acc = 0;
                for (int m = 0; m < NX; ++m) acc += Pm[i * NA + m] * sq.A[m * NX + j];
                PA[i * NX + j] = acc;
            }
            for (int j = 0; j < NU; ++j) {
                double acc = 0;
                for (int m = 0; m < NX; ++m) acc += Pm[i * NA + m] * sq.B[m * NU + j];
                acc += Pm[i * NA + NX + j];
                PB[i * NU + j] = acc;
            }
            double acc = p[i];
            for (int m = 0; m < NX; ++m) acc += Pm[i * NA + m] * sq.c[m];
            ph[i] = acc;
        }
        double Quu[NU * NU], Qux[NU * NA], qu[NU];
        for (int a = 0; a < NU; ++a) {
            for (int b = 0; b < NU; ++b) {
                double acc = sq.R[a * NU + b];
                for (int m = 0; m < NX; ++m) acc += sq.B[m * NU + a] * PB[m * NU + b];
                acc += PB[(NX + a) * NU + b];
                Quu[a * NU + b] = acc;
            }
            for (int j = 0; j < NA; ++j) {
                double acc = sq.S[j * NU + a];
                if (j < NX) {
                    for (int m = 0; m < NX; ++m) acc += sq.B[m * NU + a] * PA[m * NX + j];
                    acc += PA[(NX + a) * NX + j];
                }
                Qux[a * NA + j] = acc;
            }
            double acc = sq.r[a];
            for (int m = 0; m < NX; ++m) acc += sq.B[m * NU + a] * ph[m];
            acc += ph[NX + a];
            qu[a] = acc;
        }
        for (int a = 0; a < NU; ++a)
            for (int b = a + 1; b < NU; ++b) {
                double v = 0.5 * (Quu[a * NU + b] + Quu[b * NU + a]);
                Quu[a * NU + b] = Quu[b * NU + a] = v;
            }
        double L[20];
        if (chol4(Quu, L) != 0) return -1;
        double *K = R->Ks + k * NU * NA, *kk = R->kff + k * NU;
        for (int j = 0; j < NA; ++j) {
            double col[NU];
            for (int a = 0; a < NU; ++a) col[a] = Qux[a * NA + j];
            chol4_solve(L, col);
            for (int a = 0; a < NU; ++a) K[a * NA + j] = -col[a];
        }
        {
            double col[NU];
            for (int a = 0; a < NU; ++a) col[a] = qu[a];
            chol4_solve(L, col);
            for (int a = 0; a < NU; ++a) kk[a] = -col[a];
        }
        double Pn[NA * NA], pn[NA];
        for (int i = 0; i < NA; ++i) {
            for (int j = 0; j < NA; ++j) {
                double acc = sq.Q[i * NA + j];
                if (i < NX && j < NX)
                    for (int m = 0; m < NX; ++m) acc += sq.A[m * NX + i] * PA[m * NX + j];
                for (int a = 0; a < NU; ++a) acc += Qux[a * NA + i] * K[a * NA + j];
                Pn[i * NA + j] = acc;
            }
            double acc = sq.q[i];
            if (i < NX)
                for (int m = 0; m < NX; ++m) acc += sq.A[m * NX + i] * ph[m];
            for (int a = 0; a < NU; ++a) acc += Qux[a * NA + i] * kk[a];
            pn[i] = acc;
        }
        for (int i = 0; i < NA; ++i)
            for (int j = 0; j < NA; ++j) Pm[i * NA + j] = 0.5 * (Pn[i * NA + j] + Pn[j * NA + i]);
        memcpy(p, pn, sizeof(pn));
    }
    /* forward: du = K x~ + k, y' = A~ x~ + B~ du + c', x_{k+1} = (I + D P_xx)^-1 (y'_x - D (P_xv du + p_x)),
     * lam+_k = (P_{k+1} x~_{k+1} + p_{k+1})_x, then dp, dn */
    double xa[NA];
    memset(xa, 0, sizeof(xa));
    memset(W->dx, 0, sizeof(double) * NX);
    for (int k = 0; k < N; ++k) {
        const double *K = R->Ks + k * NU * NA, *kk = R->kff + k * NU;
        build_stage_resto(P, W, R, k, delta_w, mode_lsq, &sq, Dst[k]);
        double du[NU];
        for (int a = 0; a < NU; ++a) {
            double acc = kk[a];
            for (int j = 0; j < NA; ++j) acc += K[a * NA + j] * xa[j];
            du[a] = acc;
            W->du[k * NU + a] = acc;
        }
        const double *Pk = R->Pk1[k], *pk = R->pk1[k], *s = R->sD[k];
        double b[NX];
        for (int i = 0; i < NX; ++i) {
            double y = sq.c[i];
            for (int m = 0; m < NX; ++m) y += sq.A[i * NX + m] * xa[m];
            for (int a = 0; a < NU; ++a) y += sq.B[i * NU + a] * du[a];
            double t = pk[i];
            for (int a = 0; a < NU; ++a) t += Pk[i * NA + NX + a] * du[a];
            b[i] = (y - Dst[k][i] * t) / s[i];            /* D^-1/2 (y' - D (P_xv du + p_x)) */
        }
        cholN_solve(NX, R->Ls[k], b);
        double xn[NA];
        for (int i = 0; i < NX; ++i) xn[i] = s[i] * b[i];
        for (int a = 0; a < NU; ++a) xn[NX + a] = du[a];
        memcpy(xa, xn, sizeof(xn));
        memcpy(W->dx + (k + 1) * NX, xn, sizeof(double) * NX);
        for (int i = 0; i < NX; ++i) {
            double acc = pk[i];
            for (int j = 0; j < NA; ++j) acc += Pk[i * NA + j] * xn[j];
            W->lamp[k * NX + i] = acc;
            const int e = k * NX + i;
            double Sp, Sn, rp, rn;
            resto_pn_terms(R, e, delta_w, mode_lsq, &Sp, &Sn, &rp, &rn);
            R->dp[e] = (acc - rp) / Sp;
            R->dn[e] = (-acc - rn) / Sn;
        }
    }
    return 0;
}

/* residual of the full restoration Newton system at (dx, du, lam+, dp, dn); writes rq / rr / rc / rp / rn and
 * returns IPOPT's residual ratio (kkt_residual's form, with the p / n rows) */
static double kkt_residual_resto(const orc_params *P, orc_ws *W, resto_t *R, double delta_w)
{
    const int N = W->N;
    stage_qp sq;
    double D[NX];
    double nres = 0, nsol = 0, nrhs = 0;
    W->refine = 0;
    R->refine = 0;
    for (int k = 0; k < N; ++k) {
        build_stage_resto(P, W, R, k, delta_w, 0, &sq, D);
        const double *dxk = W->dx + k * NX, *duk = W->du + k * NU, *lk = W->lamp + k * NX;
        for (int a = 0; a < NU; ++a) {
            double acc = sq.R[a * NU + a] * duk[a];
            if (k >= 1)
                for (int i = 0; i < NX; ++i) acc += sq.S[i * NU + a] * dxk[i];
            const double g = sq.r[a];
            acc += g;
            for (int i = 0; i < NX; ++i) acc += sq.B[i * NU + a] * lk[i];
            W->rr[k * NU + a] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(g));
            nsol = fmax(nsol, fabs(duk[a]));
        }
        double xn[NX];
        f_disc(P, W->x + k * NX, W->u + k * NU, xn);
        for (int i = 0; i < NX; ++i) {
            const int e = k * NX + i;
            const double c = xn[i] - W->x[(k + 1) * NX + i] - R->p[e] + R->n[e];
            double acc = c - W->dx[(k + 1) * NX + i] - R->dp[e] + R->dn[e];
            for (int m = 0; m < NX; ++m) acc += sq.A[i * NX + m] * dxk[m];
            for (int a = 0; a < NU; ++a) acc += sq.B[i * NU + a] * duk[a];
            W->rc[e] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(c));
            nsol = fmax(nsol, fabs(lk[i]));
            double Sp, Sn, rp, rn;
            resto_pn_terms(R, e, delta_w, 0, &Sp, &Sn, &rp, &rn);
            const double ap = Sp * R->dp[e] - lk[i] + rp, an = Sn * R->dn[e] + lk[i] + rn;
            R->rp[e] = ap;
            R->rn[e] = an;
            nres = fmax(nres, fmax(fabs(ap), fabs(an)));
            nrhs = fmax(nrhs, fmax(fabs(rp), fabs(rn)));
            nsol = fmax(nsol, fmax(fabs(R->dp[e]), fabs(R->dn[e])));
        }
        if (k >= 1) {
            for (int i = 0; i < NX; ++i) {
                double acc = sq.q[i] - W->lamp[(k - 1) * NX + i];
                for (int j = 0; j < NX; ++j) acc += sq.Q[i * NA + j] * dxk[j];
                for (int a = 0; a < NU; ++a) acc += sq.S[i * NU + a] * duk[a];
                for (int m = 0; m < NX; ++m) acc += sq.A[m * NX + i] * lk[m];
                W->rq[k * NX + i] = acc;
                nres = fmax(nres, fabs(acc));
                nrhs = fmax(nrhs, fabs(sq.q[i]));
                nsol = fmax(nsol, fabs(dxk[i]));
            }
        }
    }
    {
        double Pm[NA * NA], p[NA];
        build_terminal_resto(W, R, delta_w, 0, Pm, p);
        const double *dxN = W->dx + N * NX;
        for (int i = 0; i < NX; ++i) {
            double acc = p[i] - W->lamp[(N - 1) * NX + i];
            for (int j = 0; j < NX; ++j) acc += Pm[i * NA + j] * dxN[j];
            W->rq[N * NX + i] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(p[i]));
            nsol = fmax(nsol, fabs(dxN[i]));
        }
    }
    if (nrhs + nres == 0.0) return nres;
    return nres / (fmin(nsol, 1e6 * nrhs) + nrhs);
}

/* Newton step with IPOPT's iterative refinement (refine_loop's rule) on the restoration system */
static int newton_step_resto(const orc_params *P, orc_ws *W, resto_t *R, double delta_w)
{
    const int N = W->N;
    W->refine = 0;
    R->refine = 0;
    int rc = riccati_resto(P, W, R, delta_w, 0);
    W->sweeps++;
    if (rc != 0) return rc;
    double ratio = kkt_residual_resto(P, W, R, delta_w);
    double dx[(NMAX + 1) * NX], du[NMAX * NU], dl[NMAX * NX], dp[NMAX * NX], dn[NMAX * NX];
    for (int step = 0; step < 10; ++step) {
        if (step >= 1 && ratio <= 1e-10) break;
        memcpy(dx, W->dx, sizeof(double) * (N + 1) * NX);
        memcpy(du, W->du, sizeof(double) * N * NU);
        memcpy(dl, W->lamp, sizeof(double) * N * NX);
        memcpy(dp, R->dp, sizeof(double) * N * NX);
        memcpy(dn, R->dn, sizeof(double) * N * NX);
        W->refine = 1;
        R->refine = 1;
        riccati_resto(P, W, R, delta_w, 0);
        W->refine = 0;
        R->refine = 0;
        W->sweeps++;
        for (int i = 0; i < (N + 1) * NX; ++i) W->dx[i] = dx[i] + W->dx[i];
        for (int i = 0; i < N * NU; ++i) W->du[i] = du[i] + W->du[i];
        for (int i = 0; i < N * NX; ++i) {
            W->lamp[i] = dl[i] + W->lamp[i];
            R->dp[i] = dp[i] + R->dp[i];
            R->dn[i] = dn[i] + R->dn[i];
        }
        const double nr = kkt_residual_resto(P, W, R, delta_w);
        if (!(nr < ratio)) {
            memcpy(W->dx, dx, sizeof(double) * (N + 1) * NX);
            memcpy(W->du, du, sizeof(double) * N * NU);
            memcpy(W->lamp, dl, sizeof(double) * N * NX);
            memcpy(R->dp, dp, sizeof(double) * N * NX);
            memcpy(R->dn, dn, sizeof(double) * N * NX);
            break;
        }
        ratio = nr;
    }
    return 0;
}

/* optimality errors of the restoration problem (compute_errors' quantities, with the p / n rows) */
static void compute_errors_resto(const orc_params *P, orc_ws *W, const resto_t *R, double mu, kkt_err *E)
{
    const int N = W->N;
    double dinf = 0, pinf = 0, cmu = 0, c0 = 0, sum_mult = 0, sum_z = 0;
    double A[NX * NX], B[NX * NU];
    for (int k = 0; k < N; ++k) {
        jac_disc(P, W->x + k * NX, W->u + k * NU, A, B);
        const double *lk = W->lam + k * NX;
        for (int j = 0; j < NU; ++j) {
            double acc = R->eta * R->du2[k * NU + j] * (W->u[k * NU + j] - R->uR[k * NU + j]);
            for (int i = 0; i < NX; ++i) acc += B[i * NU + j] * lk[i];
            acc += -W->zLu[k * NU + j] + W->zUu[k * NU + j];
            dinf = fmax(dinf, fabs(acc));
            const double v = W->u[k * NU + j];
            const double sl = v - W->ulo, su = W->uhi - v, zl = W->zLu[k * NU + j], zu = W->zUu[k * NU + j];
            cmu = fmax(cmu, fmax(fabs(sl * zl - mu), fabs(su * zu - mu)));
            c0 = fmax(c0, fmax(fabs(sl * zl), fabs(su * zu)));
            sum_z += zl + zu;
        }
        double xn[NX];
        f_disc(P, W->x + k * NX, W->u + k * NU, xn);
        for (int i = 0; i < NX; ++i) {
            const int e = k * NX + i;
            pinf = fmax(pinf, fabs(xn[i] - W->x[(k + 1) * NX + i] - R->p[e] + R->n[e]));
            sum_mult += fabs(lk[i]);
            dinf = fmax(dinf, fmax(fabs(RESTO_RHO - lk[i] - R->zp[e]), fabs(RESTO_RHO + lk[i] - R->zn[e])));
            cmu = fmax(cmu, fmax(fabs(R->p[e] * R->zp[e] - mu), fabs(R->n[e] * R->zn[e] - mu)));
            c0 = fmax(c0, fmax(fabs(R->p[e] * R->zp[e]), fabs(R->n[e] * R->zn[e])));
            sum_z += R->zp[e] + R->zn[e];
        }
    }
    for (int k = 1; k <= N; ++k) {
        double g[NX];
        for (int i = 0; i < NX; ++i)
            g[i] = R->eta * R->dx2[k * NX + i] * (W->x[k * NX + i] - R->xR[k * NX + i]) - W->lam[(k - 1) * NX + i];
        if (k < N) {
            jac_disc(P, W->x + k * NX, W->u + k * NU, A, B);
            const double *lk = W->lam + k * NX;
            for (int i = 0; i < NX; ++i)
                for (int m = 0; m < NX; ++m) g[i] += A[m * NX + i] * lk[m];
        }
        for (int j = 0; j < 3; ++j) {
            g[10 + j] += -W->zLw[k * 3 + j] + W->zUw[k * 3 + j];
            const double v = W->x[k * NX + 10 + j];
            const double sl = v - W->wlo, su = W->whi - v, zl = W->zLw[k * 3 + j], zu = W->zUw[k * 3 + j];
            cmu = fmax(cmu, fmax(fabs(sl * zl - mu), fabs(su * zu - mu)));
            c0 = fmax(c0, fmax(fabs(sl * zl), fabs(su * zu)));
            sum_z += zl + zu;
        }
        for (int i = 0; i < NX; ++i) dinf = fmax(dinf, fabs(g[i]));
    }
    const double s_max = 100.0;
    const double n_z = (double)(N * NU * 2 + N * 3 * 2 + 2 * N * NX);
    const double n_mult = (double)(N * NX) + n_z;
    E->s_d = fmax(s_max, (sum_mult + sum_z) / n_mult) / s_max;
    E->s_c = fmax(s_max, sum_z / n_z) / s_max;
    E->dual_inf = dinf;
    E->primal_inf = pinf;
    E->compl_mu = cmu;
    E->compl_0 = c0;
    E->dual_inf_unscaled = dinf;
}

/* theta_R = ||c_R||_1 and phi_R = f_R - mu_R sum ln(slacks) at (x, u, p, n) + alpha (dx, du, dp, dn) */
static void merit_resto(const orc_params *P, orc_ws *W, const resto_t *R, double alpha, double *theta, double *phi,
                        int *ok)
{
    const int N = W->N;
    double th = 0, lb = 0, f = 0;
    int good = 1;
    for (int k = 0; k < N; ++k) {
        double xk[NX], uk[NU], x1[NX], xn[NX];
        for (int i = 0; i < NX; ++i) {
            xk[i] = W->x[k * NX + i] + alpha * W->dx[k * NX + i];
            x1[i] = W->x[(k + 1) * NX + i] + alpha * W->dx[(k + 1) * NX + i];
        }
        for (int j = 0; j < NU; ++j) uk[j] = W->u[k * NU + j] + alpha * W->du[k * NU + j];
        f_disc(P, xk, uk, xn);
        for (int i = 0; i < NX; ++i) {
            const int e = k * NX + i;
            const double pe = R->p[e] + alpha * R->dp[e], ne = R->n[e] + alpha * R->dn[e];
            if (!(pe > 0) || !(ne > 0)) good = 0;
            th += fabs(xn[i] - x1[i] - pe + ne);
            f += RESTO_RHO * (pe + ne);
            lb += log(pe) + log(ne);
        }
        for (int j = 0; j < NU; ++j) {
            const double d = uk[j] - R->uR[k * NU + j];
            f += 0.5 * R->eta * R->du2[k * NU + j] * d * d;
            const double sl = uk[j] - W->ulo, su = W->uhi - uk[j];
            if (!(sl > 0) || !(su > 0)) good = 0;
            lb += log(sl) + log(su);
        }
    }
    for (int k = 1; k <= N; ++k) {
        for (int i = 0; i < NX; ++i) {
            const double v = W->x[k * NX + i] + alpha * W->dx[k * NX + i];
            const double d = v - R->xR[k * NX + i];
            f += 0.5 * R->eta * R->dx2[k * NX + i] * d * d;
            if (i >= 10) {
                const double sl = v - W->wlo, su = W->whi - v;
                if (!(sl > 0) || !(su > 0)) good = 0;
                lb += log(sl) + log(su);
            }
        }
    }
    *theta = th;
    *phi = f - R->mu * lb;
    *ok = good && isfinite(*phi) && isfinite(th);
}

/* directional derivative of phi_R along (dx, du, dp, dn) */
static double gbd_resto(orc_ws *W, const resto_t *R)
{
    const int N = W->N;
    double g = 0;
    for (int k = 0; k < N; ++k) {
        for (int j = 0; j < NU; ++j) {
            const double v = W->u[k * NU + j];
            double gb, sg;
            bar_terms(v, W->ulo, W->uhi, 0, 0, R->mu, &gb, &sg);
            g += (R->eta * R->du2[k * NU + j] * (v - R->uR[k * NU + j]) + gb) * W->du[k * NU + j];
        }
        for (int i = 0; i < NX; ++i) {
            const int e = k * NX + i;
            g += (RESTO_RHO - R->mu / R->p[e]) * R->dp[e] + (RESTO_RHO - R->mu / R->n[e]) * R->dn[e];
        }
    }
    for (int k = 1; k <= N; ++k)
        for (int i = 0; i < NX; ++i) {
            const double v = W->x[k * NX + i];
            double gr = R->eta * R->dx2[k * NX + i] * (v - R->xR[k * NX + i]);
            if (i >= 10) {
                double gb, sg;
                bar_terms(v, W->wlo, W->whi, 0, 0, R->mu, &gb, &sg);
                gr += gb;
            }
            g += gr * W->dx[k * NX + i];
        }
    return g;
}

/* fraction to the boundary of the restoration direction: primal (v bounds, p, n >= 0) and dual */
static void ftb_resto(orc_ws *W, const resto_t *R, double tau, double mu, double *amax, double *az)
{
    const int N = W->N;
    double am = primal_ftb(W, tau), a_z = dual_ftb(W, tau, mu);
    for (int e = 0; e < N * NX; ++e) {
        if (R->dp[e] < 0) am = fmin(am, -tau * R->p[e] / R->dp[e]);
        if (R->dn[e] < 0) am = fmin(am, -tau * R->n[e] / R->dn[e]);
        const double dzp = mu / R->p[e] - R->zp[e] - R->zp[e] / R->p[e] * R->dp[e];
        const double dzn = mu / R->n[e] - R->zn[e] - R->zn[e] / R->n[e] * R->dn[e];
        if (dzp < 0) a_z = fmin(a_z, -tau * R->zp[e] / dzp);
        if (dzn < 0) a_z = fmin(a_z, -tau * R->zn[e] / dzn);
    }
    *amax = am;
    *az = a_z;
}

/* accept a restoration step: v, lam and p, n with alpha, bound multipliers with az, kappa_sigma safeguard */
static void take_step_resto(orc_ws *W, resto_t *R, double alpha, double az, double mu)
{
    const int N = W->N;
    for (int e = 0; e < N * NX; ++e) {
        const double zp = R->zp[e] + az * (mu / R->p[e] - R->zp[e] - R->zp[e] / R->p[e] * R->dp[e]);
        const double zn = R->zn[e] + az * (mu / R->n[e] - R->zn[e] - R->zn[e] / R->n[e] * R->dn[e]);
        R->p[e] += alpha * R->dp[e];
        R->n[e] += alpha * R->dn[e];
        R->zp[e] = fmax(fmin(zp, 1e10 * mu / R->p[e]), mu / (1e10 * R->p[e]));
        R->zn[e] = fmax(fmin(zn, 1e10 * mu / R->n[e]), mu / (1e10 * R->n[e]));
    }
    take_step(W, alpha, az, mu, 1);
}

/* theta and the barrier objective of the ORIGINAL problem at the current iterate (barrier parameter mu_o) */
static void merit_orig(const orc_params *P, const orc_inst *I, orc_ws *W, double mu_o, double *theta, double *phi,
                       int *ok)
{
    eval_merit(P, I, W, W->x, W->u, mu_o, theta, phi, ok);
}

/* IPOPT FilterLSAcceptor::IsAcceptableToCurrentFilter */
static int filter_ok(double th, double ph, const double *filt_t, const double *filt_p, int nfilt)
{
    for (int f = 0; f < nfilt; ++f)
        if (!(th <= filt_t[f] || ph <= filt_p[f])) return 0;
    return 1;
}

static void filter_add(double th0, double ph0, double *filt_t, double *filt_p, int *nfilt)
{
    const double nt = (1.0 - 1e-5) * th0, np = ph0 - 1e-8 * th0;
    int w = 0;
    for (int f = 0; f < *nfilt; ++f)
        if (!(filt_t[f] >= nt && filt_p[f] >= np)) {
            filt_t[w] = filt_t[f];
            filt_p[w] = filt_p[f];
            w++;
        }
    if (w < FILTER_MAX) {
        filt_t[w] = nt;
        filt_p[w] = np;
        w++;
    }
    *nfilt = w;
}

/* The restoration phase from the current iterate (original barrier parameter mu_o, original filter with the
 * start point already added).  Returns 0 when an iterate acceptable to the original problem was found (W holds it,
 * with the multipliers reset as IPOPT does), else the final status (ST_RESTO_FAIL, ST_INFEASIBLE, ST_MAXITER;
 * W is then back at the start point).  *iters_left is decremented per restoration iteration. */
static int orc_restoration(const orc_params *P, const orc_inst *I, orc_ws *W, double mu_o, double th_ref,
                           double ph_ref, const double *ofilt_t, const double *ofilt_p, int onfilt, int *iters_left)
{
    const int N = W->N;
    resto_t *R = (resto_t *)calloc(1, sizeof(resto_t));
    orc_ws *W0 = (orc_ws *)malloc(sizeof(orc_ws));
    memcpy(W0, W, sizeof(orc_ws));
    /* reference point, D_R^2 = min(1, 1/|v_R|)^2, mu_R = max(mu, ||c||_inf) */
    double cmax = 0;
    for (int k = 0; k < N; ++k) {
        double xn[NX];
        f_disc(P, W->x + k * NX, W->u + k * NU, xn);
        for (int i = 0; i < NX; ++i) cmax = fmax(cmax, fabs(xn[i] - W->x[(k + 1) * NX + i]));
    }
    memcpy(R->xR, W->x, sizeof(double) * (N + 1) * NX);
    memcpy(R->uR, W->u, sizeof(double) * N * NU);
    for (int e = NX; e < (N + 1) * NX; ++e) {
        const double d = fmin(1.0, 1.0 / fabs(R->xR[e]));
        R->dx2[e] = d * d;
    }
    for (int e = 0; e < N * NU; ++e) {
        const double d = fmin(1.0, 1.0 / fabs(R->uR[e]));
        R->du2[e] = d * d;
    }
    double mu = fmax(mu_o, cmax);
    R->mu = mu;
    R->eta = eta_of(mu);
    /* p, n from the barrier first-order conditions given c (RestoIterateInitializer), z_p = mu / p, z_n = mu / n */
    for (int k = 0; k < N; ++k) {
        double xn[NX];
        f_disc(P, W->x + k * NX, W->u + k * NU, xn);
        for (int i = 0; i < NX; ++i) {
            const int e = k * NX + i;
            const double c = xn[i] - W->x[(k + 1) * NX + i];
            const double a = (mu - RESTO_RHO * c) / (2.0 * RESTO_RHO);
            const double n = a + sqrt(a * a + mu * c / (2.0 * RESTO_RHO));
            R->n[e] = n;
            R->p[e] = c + n;
            R->zp[e] = mu / R->p[e];
            R->zn[e] = mu / R->n[e];
        }
    }
    for (int e = 0; e < N * NU; ++e) {
        W->zLu[e] = fmin(RESTO_RHO, W->zLu[e]);
        W->zUu[e] = fmin(RESTO_RHO, W->zUu[e]);
    }
    for (int e = 3; e < (N + 1) * 3; ++e) {
        W->zLw[e] = fmin(RESTO_RHO, W->zLw[e]);
        W->zUw[e] = fmin(RESTO_RHO, W->zUw[e]);
    }
    /* constraint multipliers: least-squares estimate (constr_mult_init_max = 1000) */
    memset(W->lam, 0, sizeof(double) * N * NX);
    W->refine = 0;
    R->refine = 0;
    if (riccati_resto(P, W, R, 0.0, 1) == 0) {
        double mx = 0;
        for (int e = 0; e < N * NX; ++e) mx = fmax(mx, fabs(W->lamp[e]));
        if (mx <= 1e3) memcpy(W->lam, W->lamp, sizeof(double) * N * NX);
    }
    W->sweeps++;
    double tau = fmax(0.99, 1.0 - mu);
    double filt_t[FILTER_MAX], filt_p[FILTER_MAX];
    int nfilt = 0;
    double theta_max = -1, theta_min = -1, dw_last = 0.0;
    int status = ST_MAXITER;
    const double eps = 2.220446049250313e-16;
    for (;;) {
        kkt_err E;
        compute_errors_resto(P, W, R, mu, &E);
        const double e0 = err_value(&E, 0);
        if (!isfinite(e0)) { status = ST_NONFINITE; break; }
        if (e0 <= P->tol) {
            /* the restoration problem converged without a point the original filter accepts: IPOPT reports a
             * restoration failure when the original ||c||_inf is at most resto_failure_feasibility_threshold (its
             * documented default 1e2 tol), local infeasibility otherwise */
            double cm = 0;
            for (int k = 0; k < N; ++k) {
                double xn[NX];
                f_disc(P, W->x + k * NX, W->u + k * NU, xn);
                for (int i = 0; i < NX; ++i) cm = fmax(cm, fabs(xn[i] - W->x[(k + 1) * NX + i]));
            }
            status = (cm <= 1e2 * P->tol) ? ST_RESTO_FAIL : ST_INFEASIBLE;
            break;
        }
        if (*iters_left <= 0) { status = ST_MAXITER; break; }
        {
            const double mu_min = P->tol / 10.0;
            for (;;) {
                if (!(err_value(&E, 1) <= 10.0 * mu)) break;
                const double nmu = fmax(mu_min, fmin(0.2 * mu, pow15(mu)));
                if (nmu == mu) break;
                mu = nmu;
                R->mu = mu;
                R->eta = eta_of(mu);
                tau = fmax(0.99, 1.0 - mu);
                nfilt = 0;
                compute_errors_resto(P, W, R, mu, &E);
            }
        }
        /* direction with inertia correction */
        double dw = 0.0;
        int rc = newton_step_resto(P, W, R, 0.0);
        if (rc != 0) {
            dw = (dw_last == 0.0) ? 1e-4 : fmax(1e-20, dw_last / 3.0);
            for (;;) {
                rc = newton_step_resto(P, W, R, dw);
                if (rc == 0) { dw_last = dw; break; }
                dw *= (dw_last == 0.0) ? 100.0 : 8.0;
                if (dw > 1e40) break;
            }
            if (rc != 0) { status = ST_REG_FAIL; break; }
        }
        double amax, az;
        ftb_resto(W, R, tau, mu, &amax, &az);
        double th0, ph0;
        int ok0;
        merit_resto(P, W, R, 0.0, &th0, &ph0, &ok0);
        const double gBD = gbd_resto(W, R);
        if (theta_max < 0) {
            theta_max = 1e4 * fmax(1.0, th0);
            theta_min = 1e-4 * fmax(1.0, th0);
        }
        double amin_base = 1e-5;
        if (gBD < 0) {
            amin_base = fmin(1e-5, 1e-8 * th0 / (-gBD));
            if (th0 <= theta_min) amin_base = fmin(amin_base, pow(th0, 1.1) / pow(-gBD, 2.3));
        }
        const double alpha_min = 0.05 * amin_base;
        double alpha = amax, tht = 0, pht = 0;
        int accepted = 0;
        for (;;) {
            int okt;
            merit_resto(P, W, R, alpha, &tht, &pht, &okt);
            W->trials++;
            if (ls_accept(alpha, tht, pht, okt, th0, ph0, gBD, theta_max, theta_min, filt_t, filt_p, nfilt)) {
                accepted = 1;
                break;
            }
            alpha *= 0.5;
            if (alpha < alpha_min || !(alpha > 0.0)) break;   /* alpha_min = 0 (theta_R = 0) must still end */
        }
        if (!accepted) { status = ST_RESTO_FAIL; break; }
        {
            const int ftype = (gBD < 0) && (alpha * pow(-gBD, 2.3) > pow(th0, 1.1));
            const int armijo = (pht - ph0 - 1e-8 * alpha * gBD) <= 10.0 * eps * fabs(ph0);
            if (!ftype || !armijo) filter_add(th0, ph0, filt_t, filt_p, &nfilt);
        }
        take_step_resto(W, R, alpha, az, mu);
        W->iters++;
        (*iters_left)--;
#ifdef ORC_RTRACE
        fprintf(stderr, "  resto %4d mu %.2e E0 %.3e [d %.2e p %.2e c %.2e] thR %.3e phR %.6e gBD %.2e amax %.2e az %.2e "
                "alpha %.2e dw %.1e nf %d\n", W->iters, mu, e0, E.dual_inf / E.s_d, E.primal_inf, E.compl_0 / E.s_c,
                th0, ph0, gBD, amax, az, alpha, dw, nfilt);
#endif
        /* back to the original problem? (RestoConvergenceCheck / RestoFilterConvergenceCheck::TestOrigProgress) */
        double tho, pho;
        int oko;
        merit_orig(P, I, W, mu_o, &tho, &pho, &oko);
        if (oko && tho <= 0.9 * th_ref && filter_ok(tho, pho, ofilt_t, ofilt_p, onfilt) &&
            ((tho - (1.0 - 1e-5) * th_ref) <= 10.0 * eps * fabs(th_ref) ||
             (pho - ph_ref + 1e-8 * th_ref) <= 10.0 * eps * fabs(ph_ref))) {
            status = 0;
            break;
        }
    }
    if (status == 0) {
        /* bound multipliers from the restoration problem, reset to 1 when one exceeds 1000; lam = 0 */
        double zmax = 0;
        for (int e = 0; e < N * NU; ++e) zmax = fmax(zmax, fmax(W->zLu[e], W->zUu[e]));
        for (int e = 3; e < (N + 1) * 3; ++e) zmax = fmax(zmax, fmax(W->zLw[e], W->zUw[e]));
        if (zmax > 1e3) {
            for (int e = 0; e < N * NU; ++e) W->zLu[e] = W->zUu[e] = 1.0;
            for (int e = 3; e < (N + 1) * 3; ++e) W->zLw[e] = W->zUw[e] = 1.0;
        }
        memset(W->lam, 0, sizeof(double) * N * NX);
    } else {
        /* the solve ends at the point where the restoration started (the original problem's current iterate) */
        const int it = W->iters, sw = W->sweeps, tr = W->trials;
        memcpy(W, W0, sizeof(orc_ws));
        W->iters = it; W->sweeps = sw; W->trials = tr;
    }
    free(W0);
    free(R);
    return status;
}

/* IPOPT's watchdog procedure (BacktrackingLineSearch::StartWatchDog / StopWatchDog): the iterate and search
 * direction where it started, with that point's merit and directional derivative (FilterLSAcceptor::StartWatchDog) */
typedef struct {
    double x[(NMAX + 1) * NX], u[NMAX * NU], lam[NMAX * NX];
    double zLu[NMAX * NU], zUu[NMAX * NU], zLw[(NMAX + 1) * 3], zUw[(NMAX + 1) * 3];
    double dx[(NMAX + 1) * NX], du[NMAX * NU], lamp[NMAX * NX];
    double th, ph, gBD;
} watchdog_t;

static void wd_copy(int N, watchdog_t *D, orc_ws *W, int save)
{
#define WD_MV(f, n) (save ? memcpy(D->f, W->f, sizeof(double) * (n)) : memcpy(W->f, D->f, sizeof(double) * (n)))
    WD_MV(x, (N + 1) * NX); WD_MV(u, N * NU); WD_MV(lam, N * NX);
    WD_MV(zLu, N * NU); WD_MV(zUu, N * NU); WD_MV(zLw, (N + 1) * 3); WD_MV(zUw, (N + 1) * 3);
    WD_MV(dx, (N + 1) * NX); WD_MV(du, N * NU); WD_MV(lamp, N * NX);
#undef WD_MV
}

/* IPOPT DoBacktrackingLineSearch on the current direction: trial points alpha_max, alpha_max / 2, ... down to
 * alpha_min, second-order corrections on a rejected first trial point that did not reduce theta.  skip_first = 1:
 * start at alpha_max / 2 (the watchdog's full step from this point was already rejected); 2: start at alpha_max
 * without second-order corrections (the point is the watchdog's stored one, the factorisation is another point's).
 * Returns accepted; *n_steps = rejected trials. */
static int backtrack(const orc_params *P, const orc_inst *I, orc_ws *W, double mu, double tau, double delta_w,
                     double amax, double th0, double ph0, double gBD, double theta_max, double theta_min,
                     const double *filt_t, const double *filt_p, int nfilt, int skip_first, double *alpha_out,
                     double *alpha_test_out, double *tht, double *pht, int *soc_taken, int *n_steps_out)
{
    const int N = W->N;
    double amin_base = 1e-5;
    if (gBD < 0) {
        amin_base = fmin(1e-5, 1e-8 * th0 / (-gBD));
        if (th0 <= theta_min) amin_base = fmin(amin_base, pow(th0, 1.1) / pow(-gBD, 2.3));
    }
    const double alpha_min = 0.05 * amin_base;
    double alpha = (skip_first == 1) ? 0.5 * amax : amax;
    int accepted = 0, n_steps = 0;
    for (;; ++n_steps) {
        int okt;
        trial_merit(P, I, W, alpha, mu, tht, pht, &okt);
        if (ls_accept(alpha, *tht, *pht, okt, th0, ph0, gBD, theta_max, theta_min, filt_t, filt_p, nfilt)) {
            accepted = 1;
            *alpha_test_out = alpha;
            break;
        }
        /* second-order correction on the rejected first trial point when it did not reduce the constraint
         * violation (max_soc, kappa_soc = 0.99); acceptance is judged with the original step size */
        if (n_steps == 0 && !skip_first && okt && P->max_soc > 0 && th0 <= *tht) {
            double sdx[(NMAX + 1) * NX], sdu[NMAX * NU], slp[NMAX * NX];
            memcpy(sdx, W->dx, sizeof(double) * (N + 1) * NX);
            memcpy(sdu, W->du, sizeof(double) * N * NU);
            memcpy(slp, W->lamp, sizeof(double) * N * NX);
            trial_defects(P, W, 0.0, W->cs);
            double alpha_soc = alpha, theta_trial = *tht, theta_old = 0.0, ct[NMAX * NX];
            double sratios[4];
            int cnt = 0, sacc = 0;
            while (cnt < P->max_soc && !sacc && (cnt == 0 || theta_trial <= 0.99 * theta_old)) {
                theta_old = theta_trial;
                trial_defects(P, W, alpha_soc, ct);
                for (int e = 0; e < N * NX; ++e) W->cs[e] = alpha_soc * W->cs[e] + ct[e];
                soc_direction(P, I, W, delta_w, sratios);
                alpha_soc = primal_ftb(W, tau);
                int oks;
                trial_merit(P, I, W, alpha_soc, mu, tht, pht, &oks);
                sacc = ls_accept(alpha, *tht, *pht, oks, th0, ph0, gBD, theta_max, theta_min, filt_t, filt_p, nfilt);
                if (!sacc) {
                    cnt++;
                    theta_trial = *tht;
                }
            }
            if (sacc) {
                accepted = 1;
                *soc_taken = 1;
                *alpha_test_out = alpha;
                alpha = alpha_soc;
                W->socs++;
                break;
            }
            memcpy(W->dx, sdx, sizeof(double) * (N + 1) * NX);
            memcpy(W->du, sdu, sizeof(double) * N * NU);
            memcpy(W->lamp, slp, sizeof(double) * N * NX);
        }
        alpha *= 0.5;
        if (alpha < alpha_min) break;
    }
    *alpha_out = alpha;
    *n_steps_out = n_steps;
    return accepted;
}

/* ---- main solve ------------------------------------------------------------------------- */
static int orc_ipm(const orc_params *P, const orc_inst *I, orc_ws *W)
{
    const int N = W->N;
    /* bounds relaxed by bound_relax_factor (IPOPT default 1e-8) */
    W->ulo = P->u_lb - P->bound_relax * fmax(1.0, fabs(P->u_lb));
    W->uhi = P->u_ub + P->bound_relax * fmax(1.0, fabs(P->u_ub));
    W->wlo = P->w_lb - P->bound_relax * fmax(1.0, fabs(P->w_lb));
    W->whi = P->w_ub + P->bound_relax * fmax(1.0, fabs(P->w_ub));
    /* initial point (quad_OC.py:125-158): X0 = ini_state, U = bound midpoint, X_k = 0 */
    memset(W->x, 0, sizeof(double) * (N + 1) * NX);
    for (int i = 0; i < NX; ++i) W->x[i] = I->ini[i];
    for (int k = 0; k < N * NU; ++k) W->u[k] = 0.5 * (P->u_lb + P->u_ub);
    for (int k = 1; k <= N; ++k)
        for (int j = 0; j < 3; ++j) W->x[k * NX + 10 + j] = 0.5 * (P->w_lb + P->w_ub);
    /* IPOPT bound push (bound_push = bound_frac = 1e-2) */
    {
        double pl = fmin(1e-2 * fmax(1.0, fabs(W->ulo)), 1e-2 * (W->uhi - W->ulo));
        double pu = fmin(1e-2 * fmax(1.0, fabs(W->uhi)), 1e-2 * (W->uhi - W->ulo));
        for (int k = 0; k < N * NU; ++k) {
            if (W->u[k] < W->ulo + pl) W->u[k] = W->ulo + pl;
            if (W->u[k] > W->uhi - pu) W->u[k] = W->uhi - pu;
        }
        pl = fmin(1e-2 * fmax(1.0, fabs(W->wlo)), 1e-2 * (W->whi - W->wlo));
        pu = fmin(1e-2 * fmax(1.0, fabs(W->whi)), 1e-2 * (W->whi - W->wlo));
        for (int k = 1; k <= N; ++k)
            for (int j = 0; j < 3; ++j) {
                double *v = &W->x[k * NX + 10 + j];
                if (*v < W->wlo + pl) *v = W->wlo + pl;
                if (*v > W->whi - pu) *v = W->whi - pu;
            }
    }
    for (int k = 0; k <= N; ++k) W->wk[k] = stage_weight(P, k, I->t);
    /* attitude forms */
    dir_cosine(I->qtra, W->at.Rt);
    attitude_form(W->at.Rt, W->at.St);
    {
        double qg[4] = {1, 0, 0, 0};  /* goal_atti = [0,[1,0,0]] (quad_model.py:122,175) */
        dir_cosine(qg, W->at.Rg);
        attitude_form(W->at.Rg, W->at.Sg);
    }
    /* gradient-based objective scaling (nlp_scaling_max_gradient = 100) */
    W->s_obj = 1.0;
    {
        double gmax = 0, g[NX];
        for (int k = 1; k <= N; ++k) {
            grad_x(P, I, W, k, g);
            for (int i = 0; i < NX; ++i) gmax = fmax(gmax, fabs(g[i]));
        }
        for (int k = 0; k < N; ++k) {
            grad_u(P, I, W, k, g);
            for (int j = 0; j < NU; ++j) gmax = fmax(gmax, fabs(g[j]));
        }
        if (gmax > 100.0) W->s_obj = fmax(100.0 / gmax, 1e-8);
    }
    /* bound multipliers = 1, constraint multipliers by least squares */
    for (int k = 0; k < N * NU; ++k) W->zLu[k] = W->zUu[k] = 1.0;
    for (int k = 0; k < (N + 1) * 3; ++k) W->zLw[k] = W->zUw[k] = (k >= 3) ? 1.0 : 0.0;
    memset(W->lam, 0, sizeof(double) * N * NX);
    W->mu = P->mu_init;
    W->iters = W->sweeps = W->trials = W->refines = W->socs = W->restos = 0;
    W->refine = 0;
    W->soc = 0;
    if (P->lsq_mult_init) {
        if (riccati_solve(P, I, W, 0.0, 1) == 0) {
            double mx = 0;
            for (int i = 0; i < N * NX; ++i) mx = fmax(mx, fabs(W->lamp[i]));
            if (mx <= 1e3) memcpy(W->lam, W->lamp, sizeof(double) * N * NX);
        }
        W->sweeps++;
    }

    double mu = W->mu;
    double tau = fmax(0.99, 1.0 - mu);
    double filt_t[FILTER_MAX], filt_p[FILTER_MAX];
    int nfilt = 0;
    double theta_max = -1, theta_min = -1;
    double delta_w_last = 0.0;
    int acc_count = 0;
    int status = ST_MAXITER;
    int tiny_flag = 0;
    const double eps_tiny = 10.0 * 2.220446049250313e-16;
    int in_soft_resto = 0, soft_resto_counter = 0;   /* IPOPT soft restoration phase (try_soft_resto) */
    /* watchdog: active flag, successive shortened iterations, trial iterations taken, stored point */
    int in_wd = 0, wd_short = 0, wd_trial = 0;
    watchdog_t *wd = (P->watchdog > 0) ? (watchdog_t *)malloc(sizeof(watchdog_t)) : NULL;

    for (int it = 0; it <= P->max_iter; ++it) {
        kkt_err E;
        compute_errors(P, I, W, mu, &E);
        double e0 = err_value(&E, 0);
        W->fin_err = e0;
        W->fin_dual = E.dual_inf_unscaled;
        W->fin_primal = E.primal_inf;
        W->fin_compl = E.compl_0 / W->s_obj;
        if (!isfinite(e0)) { status = ST_NONFINITE; break; }
        /* convergence (IPOPT: tol + dual_inf_tol 1, constr_viol_tol 1e-4, compl_inf_tol 1e-4 unscaled) */
        if (e0 <= P->tol && E.dual_inf_unscaled <= 1.0 && E.primal_inf <= 1e-4 &&
            E.compl_0 / W->s_obj <= 1e-4) {
            status = ST_SOLVED;
            break;
        }
        if (e0 <= P->acceptable_tol && E.dual_inf_unscaled <= 1e10 && E.primal_inf <= 1e-2 &&
            E.compl_0 / W->s_obj <= 1e-2) {
            if (++acc_count >= P->acceptable_iter) { status = ST_ACCEPTABLE; break; }
        } else {
            acc_count = 0;
        }
        if (it == P->max_iter) { status = ST_MAXITER; break; }
        /* monotone barrier update */
        {
            double mu_min = P->tol / 10.0;
            for (;;) {
                double emu = err_value(&E, 1);
                if (!(emu <= 10.0 * mu || tiny_flag)) break;
                double nmu = fmax(mu_min, fmin(0.2 * mu, pow15(mu)));
                if (nmu == mu) {
                    if (tiny_flag) status = ST_TINY;
                    break;
                }
                mu = nmu;
                tau = fmax(0.99, 1.0 - mu);
                /* a new barrier problem resets the line search (BacktrackingLineSearch::Reset): empty filter, no
                 * soft restoration phase, watchdog off with its stored point released */
                nfilt = 0;
                in_soft_resto = 0;
                in_wd = 0;
                wd_short = 0;
                tiny_flag = 0;
                compute_errors(P, I, W, mu, &E);
            }
            if (status == ST_TINY) break;
            W->mu = mu;
        }
        /* search direction with inertia correction */
        double delta_w = 0.0;
        double ratios[4] = {0, 0, 0, 0};
        double *dpre = (W->dump && it == W->dump_it && !W->dump_refine) ? W->dump : NULL;
        int rc = newton_step(P, I, W, 0.0, ratios, dpre);
        if (rc != 0) {
            delta_w = (delta_w_last == 0.0) ? 1e-4 : fmax(1e-20, delta_w_last / 3.0);
            for (;;) {
                rc = newton_step(P, I, W, delta_w, ratios, dpre);
                if (rc == 0) { delta_w_last = delta_w; break; }
                delta_w *= (delta_w_last == 0.0) ? 100.0 : 8.0;
                if (delta_w > 1e40) break;
            }
            if (rc != 0) { status = ST_REG_FAIL; break; }
        }
        if (W->dump && it == W->dump_it && W->dump_refine) dump_step(W, W->dump);
        /* fraction-to-boundary (primal) and alpha_z */
        double amax = primal_ftb(W, tau), az = dual_ftb(W, tau, mu);
        /* current merit and directional derivative */
        double th0, ph0;
        int ok0;
        eval_merit(P, I, W, W->x, W->u, mu, &th0, &ph0, &ok0);
        const double j0 = W->mJ, lb0 = W->mlb;   /* debug trace */
        double gBD = 0;
        for (int k = 0; k < N; ++k) {
            double g[NU];
            grad_u(P, I, W, k, g);
            for (int j = 0; j < NU; ++j) {
                double gb, sg;
                bar_terms(W->u[k * NU + j], W->ulo, W->uhi, 0, 0, mu, &gb, &sg);
                gBD += (g[j] + gb) * W->du[k * NU + j];
            }
        }
        for (int k = 1; k <= N; ++k) {
            double g[NX];
            grad_x(P, I, W, k, g);
            for (int j = 0; j < 3; ++j) {
                double gb, sg;
                bar_terms(W->x[k * NX + 10 + j], W->wlo, W->whi, 0, 0, mu, &gb, &sg);
                g[10 + j] += gb;
            }
            for (int i = 0; i < NX; ++i) gBD += g[i] * W->dx[k * NX + i];
        }
        if (theta_max < 0) {
            theta_max = 1e4 * fmax(1.0, th0);
            theta_min = 1e-4 * fmax(1.0, th0);
        }
        /* tiny step test */
        double rel = 0;
        for (int k = 0; k < N * NU; ++k) rel = fmax(rel, fabs(W->du[k]) / (1.0 + fabs(W->u[k])));
        for (int k = NX; k < (N + 1) * NX; ++k) rel = fmax(rel, fabs(W->dx[k]) / (1.0 + fabs(W->x[k])));
        int accepted = 0, soc_taken = 0;
        /* IPOPT DetectTinyStep: relative step below 10 eps and constraint violation <= 1e-4 */
        int is_tiny = (rel < eps_tiny) && (th0 <= 1e-4);
        /* reference point of the acceptance tests (FilterLSAcceptor::InitThisLineSearch): the current iterate, or
         * while the watchdog is active the point where it started */
        double rth = th0, rph = ph0, rgBD = gBD;
        int skip_first = 0;
        if (in_wd && is_tiny) {
            /* a tiny step ends the watchdog: back to its stored point and direction, regular line search there */
            wd_copy(N, wd, W, 0);
            in_wd = 0;
            wd_short = 0;
            rth = th0 = wd->th;
            rph = ph0 = wd->ph;
            rgBD = gBD = wd->gBD;
            amax = primal_ftb(W, tau);
            az = dual_ftb(W, tau, mu);
            is_tiny = 0;
            skip_first = 2;
        }
        if (wd && !in_wd && !is_tiny && !in_soft_resto && wd_short >= P->watchdog) {
            wd_copy(N, wd, W, 1);   /* StartWatchDog */
            wd->th = th0;
            wd->ph = ph0;
            wd->gBD = gBD;
            wd_trial = 0;
            in_wd = 1;
        }
        double alpha = amax, alpha_test = amax;
        double tht = 0, pht = 0;
        int soft_step = 0, wd_step = 0, n_steps = 0;
        if (is_tiny) {
            accepted = 1;
            tiny_flag = 1;
        } else if (in_soft_resto) {
            /* inside the soft restoration phase: only soft steps, at most max_soft_resto_iters (10) of them */
            if (++soft_resto_counter <= 10) {
                int orig = 0;
                double as;
                if (try_soft_resto(P, I, W, mu, amax, az, th0, ph0, gBD, theta_max, theta_min, filt_t, filt_p, nfilt,
                                   &as, &orig, &tht, &pht)) {
                    accepted = 1;
                    soft_step = 1 + orig;
                    alpha = az = alpha_test = as;
                    if (orig) { in_soft_resto = 0; soft_resto_counter = 0; }
                }
            }
        } else {
            if (in_wd) {
                /* watchdog trial: the full step only, judged against the watchdog's reference point; rejected, it is
                 * still taken (no filter update) for watchdog_trial_iter_max (3) iterations, then the stored point
                 * is resumed with a regular line search that skips the full step */
                rth = wd->th;
                rph = wd->ph;
                rgBD = wd->gBD;
                int okt;
                trial_merit(P, I, W, amax, mu, &tht, &pht, &okt);
                if (ls_accept(amax, tht, pht, okt, rth, rph, rgBD, theta_max, theta_min, filt_t, filt_p, nfilt)) {
                    accepted = 1;
                    in_wd = 0;
                } else if (++wd_trial > 3) {
                    wd_copy(N, wd, W, 0);   /* StopWatchDog */
                    in_wd = 0;
                    wd_short = 0;
                    rth = th0 = wd->th;
                    rph = ph0 = wd->ph;
                    rgBD = gBD = wd->gBD;
                    amax = primal_ftb(W, tau);
                    az = dual_ftb(W, tau, mu);
                    skip_first = 1;
                } else {
                    accepted = 1;
                    wd_step = 1;
                }
                alpha = alpha_test = amax;
            }
            if (!accepted)
                accepted = backtrack(P, I, W, mu, tau, delta_w, amax, th0, ph0, gBD, theta_max, theta_min, filt_t,
                                     filt_p, nfilt, skip_first, &alpha, &alpha_test, &tht, &pht, &soc_taken, &n_steps);
            if (!accepted && !is_tiny) {
                /* the backtracking failed: try the soft restoration phase first */
                int orig = 0;
                double as;
                if (try_soft_resto(P, I, W, mu, amax, az, th0, ph0, gBD, theta_max, theta_min, filt_t, filt_p, nfilt,
                                   &as, &orig, &tht, &pht)) {
                    accepted = 1;
                    soft_step = 1 + orig;
                    alpha = az = alpha_test = as;
                    if (!orig) { in_soft_resto = 1; soft_resto_counter = 0; }
                }
            }
            /* the dual step follows the accepted direction */
            if (soc_taken) az = dual_ftb(W, tau, mu);
            /* successive iterations whose first trial point was rejected trigger the watchdog; the full step a
             * stopped watchdog skips counts as rejected (IPOPT's backtracking loop advances its trial counter past it) */
            if (accepted) wd_short = (n_steps == 0 && skip_first != 1) ? 0 : wd_short + 1;
        }
        if (is_tiny || soft_step == 1 || in_soft_resto) wd_short = 0;
        /* filter update of an accepted step (a soft step the original criterion rejected leaves it alone) */
        if (accepted && !is_tiny && soft_step != 1 && !wd_step) {
            int ftype = (rgBD < 0) && (alpha_test * pow(-rgBD, 2.3) > pow(rth, 1.1));
            int armijo = (pht - rph - 1e-8 * alpha_test * rgBD) <= 10.0 * 2.220446049250313e-16 * fabs(rph);
            if (soft_step || !ftype || !armijo) {
                /* augment the filter; drop the entries the new one dominates (IPOPT Filter::AddEntry) */
                const double nt = (1.0 - 1e-5) * rth, np = rph - 1e-8 * rth;
                int w = 0;
                for (int f = 0; f < nfilt; ++f)
                    if (!(filt_t[f] >= nt && filt_p[f] >= np)) {
                        filt_t[w] = filt_t[f];
                        filt_p[w] = filt_p[f];
                        w++;
                    }
                if (w < FILTER_MAX) {
                    filt_t[w] = nt;
                    filt_p[w] = np;
                    w++;
                }
                nfilt = w;
            }
        }
        if (W->trace && it < W->trace_iters) {
            double *tr = W->trace + it * 16;
            tr[0] = mu; tr[1] = e0; tr[2] = th0; tr[3] = ph0; tr[4] = gBD; tr[5] = amax; tr[6] = az;
            tr[7] = alpha; tr[8] = delta_w; tr[9] = accepted; tr[10] = nfilt; tr[11] = W->sweeps;
            tr[12] = ratios[0]; tr[13] = ratios[1]; tr[14] = j0; tr[15] = lb0;
        }
#ifdef ORC_TRACE
        fprintf(stderr, "it %3d mu %.2e E0 %.3e [d %.2e p %.2e c %.2e sd %.2f] th %.3e ph %.10e gBD %.3e amax %.3e az %.3e alpha %.3e dw %.2e acc %d nf %d s %.3e arg %d %d %d\n",
                it, mu, e0, E.dual_inf / E.s_d, E.primal_inf, E.compl_0 / E.s_c, E.s_d, th0, ph0, gBD, amax, az, alpha, delta_w, accepted, nfilt, W->s_obj, E.arg_type, E.arg_k, E.arg_i);
        if (E.arg_type == 0) fprintf(stderr, "   u=%.17g  sl=%.3e su=%.3e zl=%.3e zu=%.3e\n", W->u[E.arg_k*NU+E.arg_i], W->u[E.arg_k*NU+E.arg_i]-W->ulo, W->uhi-W->u[E.arg_k*NU+E.arg_i], W->zLu[E.arg_k*NU+E.arg_i], W->zUu[E.arg_k*NU+E.arg_i]);
#endif
        if (!accepted) {
            /* the line search and the soft restoration phase failed.  At an almost feasible point IPOPT does not
             * restore (it returns its last acceptable point, or fails): here the current iterate counts as
             * acceptable when it meets acceptable_tol, else the solve ends as a line-search failure.  Otherwise
             * the start point enters the filter (PrepareRestoPhaseStart) and the restoration phase runs. */
            if (th0 <= 1e-2 * P->tol || !P->restoration) {
                status = (e0 <= P->acceptable_tol) ? ST_ACCEPTABLE : ST_LS_FAIL;
                break;
            }
            filter_add(th0, ph0, filt_t, filt_p, &nfilt);
            int left = P->max_iter - it;
            const int it0 = W->iters;
            const int rs = orc_restoration(P, I, W, mu, th0, ph0, filt_t, filt_p, nfilt, &left);
            W->restos++;
            it += W->iters - it0 - 1;   /* the restoration's iterations count (this one included) */
            if (rs != 0) {
                status = (rs == ST_RESTO_FAIL && e0 <= P->acceptable_tol) ? ST_ACCEPTABLE : rs;
                break;
            }
            in_soft_resto = 0;
            soft_resto_counter = 0;
            wd_short = 0;
            continue;
        }
        if (is_tiny) alpha = amax;
        /* accept: primal, lambda (alpha_for_y = primal), z (alpha_z; a soft restoration step moves all of them by
         * its alpha), then the kappa_sigma safeguard (1e10) */
        take_step(W, alpha, az, mu, 1);
        W->iters++;
    }
    free(wd);
    /* honor_original_bounds */
    for (int k = 0; k < N * NU; ++k) W->u[k] = fmin(fmax(W->u[k], P->u_lb), P->u_ub);
    for (int k = 1; k <= N; ++k)
        for (int j = 0; j < 3; ++j) {
            double *v = &W->x[k * NX + 10 + j];
            *v = fmin(fmax(*v, P->w_lb), P->w_ub);
        }
    return status;
}

/* ------------------------------------------------------------------------------------------ */
/* reward: rotor tips + collis_det (solid_geometry.py) + goal path term (quad_policy.py:67-91)  */
/* ------------------------------------------------------------------------------------------ */

/* np.dot of two float64 3-vectors: OpenBLAS ddot's tail loop, an FMA chain (verified bit-exact
 * against this image's numpy on 2e4 random vectors; tests/test_oracle_golden.py) */
static double dot3(const double *a, const double *b) { return fma(a[2], b[2], fma(a[1], b[1], a[0] * b[0])); }
/* magni(): solid_geometry.py:7-8 */
static double magni3(const double *v) { return sqrt(dot3(v, v)); }
static void cross3(const double *a, const double *b, double *c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
static void normv(const double *a, double *o)
{
    double m = magni3(a);
    o[0] = a[0] / m; o[1] = a[1] / m; o[2] = a[2] / m;
}

typedef struct { double p1[3], normal[3], vec1[3], vec2[3], n1[3], n2[3], n3[3]; } plane_t;
typedef struct { double p1[3], p2[3], dir[3]; } line_t;
typedef struct {
    double pt[4][3];
    double centroid[3];
    plane_t pl[4];
    line_t ln[4];
} obstacle_t;

/* plane(point1, point2, point3): solid_geometry.py:16-47 */
static void plane_init(plane_t *P, const double *a, const double *b, const double *c)
{
    for (int i = 0; i < 3; ++i) {
        P->p1[i] = a[i];
        P->vec1[i] = b[i] - a[i];
        P->vec2[i] = c[i] - a[i];
    }
    double cr[3];
    cross3(P->vec2, P->vec1, cr);
    normv(cr, P->normal);
    cross3(P->vec1, P->normal, cr);
    normv(cr, P->n1);
    cross3(P->normal, P->vec2, cr);
    normv(cr, P->n2);
    double v3[3] = {c[0] - b[0], c[1] - b[1], c[2] - b[2]};
    cross3(P->normal, v3, cr);
    normv(cr, P->n3);
}

/* line(point1, point2): solid_geometry.py:50-78 */
static void line_init(line_t *L, const double *a, const double *b)
{
    double d[3];
    for (int i = 0; i < 3; ++i) {
        L->p1[i] = a[i];
        L->p2[i] = b[i];
        d[i] = a[i] - b[i];
    }
    normv(d, L->dir);
}
static double line_vertical(const line_t *L, const double *pt)
{
    double d[3] = {pt[0] - L->p1[0], pt[1] - L->p1[1], pt[2] - L->p1[2]}, c[3];
    cross3(d, L->dir, c);
    return magni3(c);
}
static double line_distance(const line_t *L, const double *pt)
{
    double a = line_vertical(L, pt);
    double d1[3] = {pt[0] - L->p1[0], pt[1] - L->p1[1], pt[2] - L->p1[2]};
    double d2[3] = {pt[0] - L->p2[0], pt[1] - L->p2[1], pt[2] - L->p2[2]};
    double d3[3] = {L->p1[0] - L->p2[0], L->p1[1] - L->p2[1], L->p1[2] - L->p2[2]};
    double b = magni3(d1), c = magni3(d2), d = magni3(d3);
    if (b > c) return ((b * b - d * d) > a * a) ? c : a;
    return ((c * c - d * d) > a * a) ? b : a;
}

/* obstacle(point1..4): solid_geometry.py:82-102 */
void orc_obstacle_init(obstacle_t *O, const double *g12)
{
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j) O->pt[i][j] = g12[i * 3 + j];
    for (int j = 0; j < 3; ++j)
        O->centroid[j] = (O->pt[0][j] + O->pt[1][j] + O->pt[2][j] + O->pt[3][j]) / 4;
    for (int i = 0; i < 4; ++i) plane_init(&O->pl[i], O->centroid, O->pt[i], O->pt[(i + 1) % 4]);
    for (int i = 0; i < 4; ++i) line_init(&O->ln[i], O->pt[i], O->pt[(i + 1) % 4]);
}

/* collis_det(vert_traj, horizon): solid_geometry.py:104-168.
 * branch: 0 = starts behind plane1 / never crosses; 1+4*p+b: last matching plane p, b=0 inside, 1 edge.
 * co: 1 if the crossing is inside the gate. */
static double collis_det(const obstacle_t *O, const double *traj, int stride, int horizon, int *branch, int *co)
{
    double collision = 0;
    *co = 0;
    *branch = 0;
    const double *n0 = O->pl[0].normal;
    double d0[3];
    for (int i = 0; i < 3; ++i) d0[i] = traj[i] - O->centroid[i];
    if (dot3(n0, d0) < 0) return 0;
    const double dmin = 0.2;
    for (int t = 0; t < horizon; ++t) {
        const double *pt = traj + t * stride;
        double dd[3] = {pt[0] - O->centroid[0], pt[1] - O->centroid[1], pt[2] - O->centroid[2]};
        if (!(dot3(n0, dd) < 0)) continue;
        const double *pp = traj + ((t - 1 + (horizon + 1)) % (horizon + 1)) * stride; /* t-1, -1 wraps */
        /* interpoint (plane1): solid_geometry.py:43-47 */
        double dir[3], dv[3] = {pt[0] - pp[0], pt[1] - pp[1], pt[2] - pp[2]};
        normv(dv, dir);
        double rel[3] = {pt[0] - O->pl[0].p1[0], pt[1] - O->pl[0].p1[1], pt[2] - O->pl[0].p1[2]};
        double tt = 1 / dot3(dir, n0) * dot3(n0, rel);
        double X[3] = {pt[0] - tt * dir[0], pt[1] - tt * dir[1], pt[2] - tt * dir[2]};
        double xc[3] = {X[0] - O->centroid[0], X[1] - O->centroid[1], X[2] - O->centroid[2]};
        for (int p = 0; p < 4; ++p) {
            const plane_t *pl = &O->pl[p];
            if (dot3(pl->n1, xc) > 0 && dot3(pl->n2, xc) > 0) {
                double pv[3] = {O->pt[p][0] - X[0], O->pt[p][1] - X[1], O->pt[p][2] - X[2]};
                if (dot3(pv, pl->n3) > 0) {
                    double m = line_vertical(&O->ln[0], X);
                    for (int l = 1; l < 4; ++l) m = fmin(m, line_vertical(&O->ln[l], X));
                    double e = fmax(0.0, dmin - m);
                    collision = -(e * e);
                    *co = 1;
                    *branch = 1 + 4 * p;
                } else {
                    /* edge lines: plane1 {4,1,2}, plane2 {1,2,3}, plane3 {2,3,4}, plane4 {3,4,1} */
                    int l0 = (p + 3) % 4, l1 = p, l2 = (p + 1) % 4;
                    double m = line_distance(&O->ln[l0], X);
                    m = fmin(m, line_distance(&O->ln[l1], X));
                    m = fmin(m, line_distance(&O->ln[l2], X));
                    collision = -2 * dmin * m - dmin * dmin;
                    *branch = 2 + 4 * p;
                }
            }
        }
        break;
    }
    return collision;
}

/* rotor tips (quad_model.py:239-276) + reward (quad_policy.py:80-90) */
static double reward_from_traj(const orc_params *P, const obstacle_t *O, const double *goal, const double *x,
                               int N, int *branches)
{
    double a = P->wing_len * 0.5 / sqrt(2.0);
    double b[4][3] = {{a, a, 0}, {-a, a, 0}, {-a, -a, 0}, {a, -a, 0}};
    static const int NPT = NMAX + 1;
    double tr[4][(NMAX + 1) * 3];
    (void)NPT;
    for (int t = 0; t <= N; ++t) {
        const double *xt = x + t * NX;
        double C[9];
        dir_cosine(xt + 6, C);
        for (int r = 0; r < 4; ++r)
            for (int i = 0; i < 3; ++i)
                tr[r][t * 3 + i] = xt[i] + (C[0 * 3 + i] * b[r][0] + C[1 * 3 + i] * b[r][1] + C[2 * 3 + i] * b[r][2]);
    }
    double col = 0;
    for (int r = 0; r < 4; ++r) {
        int br, co;
        col += collis_det(O, tr[r], 3, N, &br, &co);
        if (branches) branches[r] = br;
    }
    double path = 0;
    for (int p = 0; p < 4; ++p) {
        const double *xt = x + (N - 1 - p) * NX;
        double d[3] = {xt[0] - goal[0], xt[1] - goal[1], xt[2] - goal[2]};
        path += dot3(d, d);
    }
    return 1000 * col - 0.5 * path + 100;
}

/* ------------------------------------------------------------------------------------------ */
/* exported API (ctypes)                                                                       */
/* ------------------------------------------------------------------------------------------ */

void orc_default_params(orc_params *P)
{
    memset(P, 0, sizeof(*P));
    P->mass = 0.5; P->Jx = 0.0023; P->Jy = 0.0023; P->Jz = 0.004;
    P->arm_l = 0.35; P->c_tau = 0.0245; P->grav = 9.78; P->dt = 0.1;
    P->wrt = 5; P->wqt = 80; P->wthrust = 0.1; P->wrf = 5; P->wvf = 5; P->wqf = 0; P->wwf = 3;
    P->tra_w_peak = 60; P->tra_w_decay = 10; P->du_weight = 1;
    P->u_lb = 0; P->u_ub = 2 * 1.22; P->w_lb = -3.141592653589793 / 2; P->w_ub = 3.141592653589793 / 2;
    P->wing_len = 1.5; P->d_min = 0.2;
    P->horizon = 50;
    P->max_iter = 3000; P->tol = 1e-8; P->acceptable_tol = 1e-6; P->acceptable_iter = 15;
    P->mu_init = 0.1; P->bound_relax = 1e-8; P->lsq_mult_init = 1;
    P->max_soc = 4;
    P->restoration = 1;
    P->watchdog = 10;
    P->grad_mode = 0;
}

int orc_params_size(void) { return (int)sizeof(orc_params); }
/* the barrier update's mu^1.5 (tests: correctly rounded against an exact reference) */
double orc_pow15(double x) { return pow15(x); }

static void make_inst(const double *ini, const double *goal, const double *ptra, const double *qtra, double t,
                      const double *ulast, orc_inst *I)
{
    memcpy(I->ini, ini, sizeof(double) * NX);
    memcpy(I->goal, goal, sizeof(double) * 3);
    memcpy(I->ptra, ptra, sizeof(double) * 3);
    memcpy(I->qtra, qtra, sizeof(double) * 4);
    I->t = t;
    if (ulast) memcpy(I->ulast, ulast, sizeof(double) * 4);
    else memset(I->ulast, 0, sizeof(double) * 4);
}

/* Batched forward solve on quaternion-parameterised traversal attitude.
 * x_out B x (N+1) x 13, u_out B x N x 4, lam_out B x N x 13 (unscaled lam_g), cost B.
 * counters (nullable) B x 3: iterations, Riccati sweeps, line-search trials. */
static double *g_trace = NULL;
static int g_trace_iters = 0;
static double *g_dump = NULL;
static int g_dump_it = -1, g_dump_refine = 0;
void orc_debug_trace(double *buf, int iters) { g_trace = buf; g_trace_iters = iters; }
void orc_debug_dump(double *buf, int it, int after_refine) { g_dump = buf; g_dump_it = it; g_dump_refine = after_refine; }
/* Debug: per instance 4 doubles [overall NLP error (scaled, IPOPT's convergence measure), unscaled dual
 * infeasibility, primal infeasibility, unscaled complementarity] at the last iterate of later solves */
static double *g_final_err = NULL;
void orc_debug_final_err(double *buf) { g_final_err = buf; }

int orc_solve_q(const orc_params *P, int64_t B, const double *ini, const double *goal, const double *ptra,
                const double *qtra, const double *t, const double *ulast, double *x_out, double *u_out,
                double *lam_out, double *cost, int32_t *status, int32_t *counters)
{
    const int N = P->horizon;
    if (N < 1 || N > NMAX) return -1;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t b = 0; b < B; ++b) {
        orc_ws *W = (orc_ws *)malloc(sizeof(orc_ws));
        W->N = N;
        W->trace = g_trace ? g_trace + b * (int64_t)g_trace_iters * 16 : NULL;
        W->trace_iters = g_trace_iters;
        W->dump = g_dump ? g_dump + b * (int64_t)((NMAX_DUMP + 1) * NX + NMAX_DUMP * NU + NMAX_DUMP * NX) : NULL;
        W->dump_it = g_dump_it;
        W->dump_refine = g_dump_refine;
        orc_inst I;
        make_inst(ini + b * NX, goal + b * 3, ptra + b * 3, qtra + b * 4, t[b], ulast ? ulast + b * 4 : NULL, &I);
        int st = orc_ipm(P, &I, W);
        if (status) status[b] = st;
        if (g_final_err) {
            double *fe = g_final_err + b * 4;
            fe[0] = W->fin_err; fe[1] = W->fin_dual; fe[2] = W->fin_primal; fe[3] = W->fin_compl;
        }
        if (counters) {
            counters[b * 3 + 0] = W->iters;
            counters[b * 3 + 1] = W->sweeps;
            counters[b * 3 + 2] = W->trials;
        }
        if (x_out) memcpy(x_out + b * (N + 1) * NX, W->x, sizeof(double) * (N + 1) * NX);
        if (u_out) memcpy(u_out + b * N * NU, W->u, sizeof(double) * N * NU);
        if (lam_out)
            for (int i = 0; i < N * NX; ++i) lam_out[b * N * NX + i] = W->lam[i] / W->s_obj;
        if (cost) cost[b] = objective_J(P, &I, W, W->x, W->u);
        free(W);
    }
    return 0;
}

/* Reward of given state trajectories (B x (N+1) x 13) against gates (B x 12) and goals. */
int orc_reward(const orc_params *P, int64_t B, const double *x, const double *goal, const double *gate12,
               double *reward, int32_t *branches)
{
    const int N = P->horizon;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < B; ++b) {
        obstacle_t O;
        orc_obstacle_init(&O, gate12 + b * 12);
        reward[b] = reward_from_traj(P, &O, goal + b * 3, x + b * (N + 1) * NX, N, branches ? branches + b * 4 : NULL);
    }
    return 0;
}

/* collis_det on raw tracks (tests): tracks B x (horizon+1) x 3 */
int orc_collis_det(int64_t B, int horizon, const double *gate12, const double *tracks, double *out,
                   int32_t *branch, int32_t *co)
{
    for (int64_t b = 0; b < B; ++b) {
        obstacle_t O;
        orc_obstacle_init(&O, gate12 + b * 12);
        int br, c;
        out[b] = collis_det(&O, tracks + b * (horizon + 1) * 3, 3, horizon, &br, &c);
        if (branch) branch[b] = br;
        if (co) co[b] = c;
    }
    return 0;
}

/* model evaluations for golden-vector tests: f, A, B, sum lam*Hess, costs */
int orc_model_eval(const orc_params *P, int64_t n, const double *x, const double *u, const double *lam,
                   double *f, double *A, double *Bm, double *Hxx, double *Hxu)
{
    for (int64_t i = 0; i < n; ++i) {
        const double *xi = x + i * NX, *ui = u + i * NU;
        if (f) f_cont(P, xi, ui, f + i * NX);
        if (A && Bm) jac_disc(P, xi, ui, A + i * NX * NX, Bm + i * NX * NU);
        if (Hxx && Hxu) {
            memset(Hxx + i * NX * NX, 0, sizeof(double) * NX * NX);
            memset(Hxu + i * NX * NU, 0, sizeof(double) * NX * NU);
            hess_lam_disc(P, xi, ui, lam + i * NX, Hxx + i * NX * NX, Hxu + i * NX * NU);
        }
    }
    return 0;
}

int orc_cost_eval(const orc_params *P, int64_t n, const double *x, const double *goal, const double *ptra,
                  const double *qtra, const double *wk, double *path, double *tra, double *grad, double *hess)
{
    for (int64_t i = 0; i < n; ++i) {
        att_t at;
        dir_cosine(qtra + i * 4, at.Rt);
        attitude_form(at.Rt, at.St);
        double qg[4] = {1, 0, 0, 0};
        dir_cosine(qg, at.Rg);
        attitude_form(at.Rg, at.Sg);
        const double *xi = x + i * NX;
        if (path) path[i] = path_cost(P, &at, goal + i * 3, xi);
        if (tra) tra[i] = tra_cost(P, &at, ptra + i * 3, xi);
        if (grad && hess) {
            memset(hess + i * NX * NX, 0, sizeof(double) * NX * NX);
            state_cost_derivs(P, &at, goal + i * 3, ptra + i * 3, wk[i], xi, grad + i * NX, hess + i * NX * NX);
        }
    }
    return 0;
}

/* ---- policy layer: objective / sol_gradient / get_input quirks ---------------- */

/* round(np.float32 t, 1): numpy around in float32 */
static double round1_f32(float t)
{
    volatile float y = t * 10.0f;
    float r = rintf(y);
    volatile float z = r / 10.0f;
    return (double)z;
}
/* round(np.float64 t, 1) */
static double round1_f64(double t)
{
    volatile double y = t * 10.0;
    return rint(y) / 10.0;
}
/* magni(np.float32 vector): np.dot -> OpenBLAS sdot tail loop (float products accumulated in
 * double, result rounded to float), then float32 sqrt */
static double magni_f32(const float *a)
{
    volatile float p0 = a[0] * a[0], p1 = a[1] * a[1], p2 = a[2] * a[2];
    double acc = 0.0;
    acc += (double)p0;
    acc += (double)p1;
    acc += (double)p2;
    float s = (float)acc;
    return (double)sqrtf(s);
}

/* Parameters of solve j (0..8) of sol_gradient for one sample (quad_policy.py:97-110):
 * j=0 nominal, 1..3 +delta on p, 4..6 +delta on the angle vector, 7 t-0.1, 8 t+0.1. */
static void grad_job_params(const orc_params *P, const float *o, int j, double *p, double *q, double *t,
                            int *use_ulast)
{
    const double delta = 1e-3;
    double a[3] = {(double)o[3], (double)o[4], (double)o[5]};
    for (int i = 0; i < 3; ++i) p[i] = (double)o[i];
    double anorm = magni_f32(o + 3);
    *t = round1_f32(o[6]);
    *use_ulast = (j >= 1 && j <= 6);
    if (j >= 1 && j <= 3) p[j - 1] += delta;
    if (j >= 4 && j <= 6) {
        a[j - 4] += delta;
        anorm = magni3(a);
    }
    if (j == 7) *t = P->t_probe_f32 ? round1_f32((float)(o[6] - 0.1f)) : round1_f64((double)o[6] - 0.1);
    if (j == 8) *t = P->t_probe_f32 ? round1_f32((float)(o[6] + 0.1f)) : round1_f64((double)o[6] + 0.1);
    orc_rd2quat(anorm, a, q);
}

/* out8 from the 9 rewards (quad_policy.py:97-112) */
static void assemble_one(const orc_params *P, const double *R, const float *o, double *out8)
{
    double j0 = R[0];
    double d[7];
    for (int i = 0; i < 3; ++i) {
        double v = R[1 + i] - j0;
        v = v < -0.5 ? -0.5 : (v > 0.5 ? 0.5 : v);
        d[i] = v * 0.1;
    }
    for (int i = 0; i < 3; ++i) {
        double v = R[4 + i] - j0;
        v = v < -0.5 ? -0.5 : (v > 0.5 ? 0.5 : v);
        double sc;
        if (P->t_probe_f32) {  /* NumPy >= 2: 1/(500*a**2+5) stays float32 */
            volatile float af = o[3 + i];
            volatile float a2 = af * af;
            volatile float den = 500.0f * a2;
            den = den + 5.0f;
            volatile float qq = 1.0f / den;
            sc = (double)qq;
        } else {               /* NumPy 1.23 (reference env): np.float32 ** 2 -> float64 */
            double ai = (double)o[3 + i];
            sc = 1 / (500 * (ai * ai) + 5);
        }
        d[3 + i] = v * sc;
    }
    double drdt = 0;
    if ((R[7] - j0) > 2) drdt = -0.05;
    if ((R[8] - j0) > 2) drdt = 0.05;
    d[6] = drdt;
    for (int i = 0; i < 7; ++i) out8[i] = -d[i];
    out8[7] = j0;
}

/* per-job parameters for a batch (tests): p B x 9 x 3, q B x 9 x 4, t B x 9, use_ulast B x 9 */
int orc_grad_params(const orc_params *P, int64_t B, const float *dnn_out, double *p, double *q, double *t,
                    int32_t *use_ulast)
{
    for (int64_t b = 0; b < B; ++b)
        for (int j = 0; j < 9; ++j) {
            int uu;
            grad_job_params(P, dnn_out + b * 7, j, p + (b * 9 + j) * 3, q + (b * 9 + j) * 4, t + b * 9 + j, &uu);
            if (use_ulast) use_ulast[b * 9 + j] = uu;
        }
    return 0;
}

int orc_assemble(const orc_params *P, int64_t B, const double *R9, const float *dnn_out, double *out8)
{
    for (int64_t b = 0; b < B; ++b) assemble_one(P, R9 + b * 9, dnn_out + b * 7, out8 + b * 8);
    return 0;
}

/* IFT gradient mode (grad_mode = 1; the HIP kernel's ift_probes restates the same steps).  The reference's
 * sol_gradient (quad_policy.py:99-105) re-solves the NLP at p + 1e-3 e_i and a + 1e-3 e_i; here the six perturbed
 * optima are predicted to first order from the nominal optimum z*:
 *   1. one Newton-system factorisation at z* (final barrier parameter and bound duals, delta_w = 0);
 *   2. per parameter theta_i in (p_tra, a_tra): right-hand side dF/dtheta_i, nonzero only in the x rows of stages
 *      1..N-1 where the traversal cost lives (quad_model.py:200-213): s * d(grad_x (w_k tra + path))/dtheta_i as a
 *      central difference (h = 1e-5) of the analytic gradient; the a probes rebuild the traversal attitude from
 *      a +- h e_i (Rd2Rp + toQuaternion with the float64 norm);
 *   3. dz_opt/dtheta_i = -K^-1 dF/dtheta_i with that factorisation (the refinement right-hand-side path);
 *   4. the probe reward is scored exactly on x_opt + 1e-3 dx_opt/dtheta_i (the assembly's clipping then applies to
 *      R(x* + delta dx/dtheta) - j where the FD mode has R(theta + delta e_i) - j).
 * ok = 0 (nominal not solved): every probe reward is R0. */
/* Returns 0 when the factorisation at z* met a wrong inertia: the probe rewards then fall back to R0 and the
 * caller reports their status as ST_REG_FAIL (the kernel's ift_probes does the same). */
static int orc_ift_probes(const orc_params *P, const orc_inst *I, orc_ws *W, const obstacle_t *O, const double *goal,
                          const double *a3, int ok, double R0, double *Rprobe)
{
    const int N = W->N;
    const double h = 1e-5, delta = 1e-3;
    if (!ok) {
        for (int q = 0; q < 6; ++q) Rprobe[q] = R0;
        return 1;
    }
    int fac_ok = 1;
    double xs[(NMAX + 1) * NX];
    memcpy(xs, W->x, sizeof(double) * (N + 1) * NX);
    for (int q = 0; q < 6; ++q) {
        att_t ap = W->at, am = W->at;
        double pp[3], pm[3];
        memcpy(pp, I->ptra, sizeof(pp));
        memcpy(pm, I->ptra, sizeof(pm));
        if (q < 3) {
            pp[q] += h;
            pm[q] -= h;
        } else {
            double ah[3] = {a3[0], a3[1], a3[2]}, qh[4];
            ah[q - 3] = a3[q - 3] + h;
            orc_rd2quat(magni3(ah), ah, qh);
            dir_cosine(qh, ap.Rt);
            attitude_form(ap.Rt, ap.St);
            ah[q - 3] = a3[q - 3] - h;
            orc_rd2quat(magni3(ah), ah, qh);
            dir_cosine(qh, am.Rt);
            attitude_form(am.Rt, am.St);
        }
        memset(W->rq, 0, sizeof(double) * (N + 1) * NX);
        memset(W->rr, 0, sizeof(double) * N * NU);
        memset(W->rc, 0, sizeof(double) * N * NX);
        for (int k = 1; k < N; ++k) {
            double gp[NX], gm[NX];
            state_cost_derivs(P, &ap, goal, pp, W->wk[k], xs + k * NX, gp, NULL);
            state_cost_derivs(P, &am, goal, pm, W->wk[k], xs + k * NX, gm, NULL);
            for (int i = 0; i < NX; ++i) W->rq[k * NX + i] = W->s_obj * (gp[i] - gm[i]) / (2 * h);
        }
        W->refine = 1;
        const int rc = riccati_solve(P, I, W, 0.0, 0);   /* factorises at z* and solves with rq */
        W->refine = 0;
        if (rc != 0) {
            Rprobe[q] = R0;
            fac_ok = 0;
            continue;
        }
        double xp[(NMAX + 1) * NX];
        for (int e = 0; e < (N + 1) * NX; ++e) xp[e] = xs[e] + delta * W->dx[e];
        Rprobe[q] = reward_from_traj(P, O, goal, xp, N, NULL);
    }
    return fac_ok;
}

/* sol_gradient (quad_policy.py:94-112) for a batch; dnn_out B x 7 float32 (p, a, t).
 * rewards_out (nullable) B x 9 (j, +dx,+dy,+dz,+da,+db,+dc, t-0.1, t+0.1). */
/* Debug: IPM iteration count of every sol_gradient job into buf (B x 9, rewards9 slot order; IFT-mode probe
 * slots 1..6 get the nominal's count) of later orc_sol_gradient calls.  NULL disables. */
static int32_t *g_grad_iters = NULL;
void orc_debug_grad_iters(int32_t *buf) { g_grad_iters = buf; }

int orc_sol_gradient(const orc_params *P, int64_t B, const double *ini, const double *goal, const double *gate12,
                     const float *dnn_out, const double *ulast, double *out8, double *rewards_out, int32_t *status)
{
    const int N = P->horizon;
    double *R = rewards_out ? rewards_out : (double *)malloc(sizeof(double) * 9 * (size_t)B);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t job = 0; job < B * 9; ++job) {
        int64_t b = job / 9;
        int j = (int)(job % 9);
        double p[3], q[4], t;
        int uu;
        grad_job_params(P, dnn_out + b * 7, j, p, q, &t, &uu);
        const double *ul = (uu && ulast) ? ulast + b * 4 : NULL;
        orc_ws *W = (orc_ws *)malloc(sizeof(orc_ws));
        W->N = N;
        W->trace = NULL;
        W->trace_iters = 0;
        W->dump = NULL;
        W->dump_it = -1;
        W->dump_refine = 0;
        orc_inst I;
        make_inst(ini + b * NX, goal + b * 3, p, q, t, ul, &I);
        if (P->grad_mode == 1 && j >= 1 && j <= 6) {   /* IFT: these probes come from the nominal job */
            free(W);
            continue;
        }
        int st = orc_ipm(P, &I, W);
        obstacle_t O;
        orc_obstacle_init(&O, gate12 + b * 12);
        R[b * 9 + j] = reward_from_traj(P, &O, goal + b * 3, W->x, N, NULL);
        if (status) status[b * 9 + j] = st;
        if (g_grad_iters) {
            g_grad_iters[b * 9 + j] = W->iters;
            if (P->grad_mode == 1 && j == 0)
                for (int q = 1; q <= 6; ++q) g_grad_iters[b * 9 + q] = W->iters;
        }
        if (P->grad_mode == 1 && j == 0) {
            const float *o = dnn_out + b * 7;
            const double a[3] = {(double)o[3], (double)o[4], (double)o[5]};
            const int okz = orc_ift_probes(P, &I, W, &O, goal + b * 3, a, st <= ST_ACCEPTABLE, R[b * 9], R + b * 9 + 1);
            if (status)
                for (int q = 1; q <= 6; ++q) status[b * 9 + q] = (st <= ST_ACCEPTABLE && !okz) ? ST_REG_FAIL : st;
        }
        free(W);
    }
    if (out8)
        for (int64_t b = 0; b < B; ++b) assemble_one(P, R + b * 9, dnn_out + b * 7, out8 + b * 8);
    if (!rewards_out) free(R);
    return 0;
}

int orc_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* threads of the OpenMP loops (bench.py's 1-core cpu_baseline); n <= 0 leaves the setting unchanged */
void orc_set_num_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
