// lane_kernel.hip — lane-per-instance interior-point solve of the quad_OC NLP on CDNA4 (gfx950).
//
// One LANE owns one NLP instance (64 independent instances per wavefront); there is no cross-lane
// traffic at all, so every VALU slot does useful work and the only synchronisation is the wave's own
// s_waitcnt.  Algorithm: identical to ipm_kernel.hip / oracle/lafse3_oracle.c (IPOPT-style primal-dual
// barrier method, filter line search, inertia correction, iterative refinement), restated as per-lane
// sequential loops over the horizon.
//
// Memory layout (HBM workspace, per wave block of 64 instances): slot-major, lane-minor —
// element `slot` of the lane's instance lives at block_base + (slot * 64 + lane) * 8, so every
// per-lane access of one slot by the wave is one contiguous 512-byte transaction.  Slots: the
// trajectories (x, u, lambda, bound duals, Newton step, refinement corrections / right-hand sides,
// stage weights) and the Riccati factors P_{k+1} (packed 17x17 upper, 153), K_k (4x17), k_k, chol(Quu_k).
// Per-instance constants (attitude forms, goal, traversal point, u_last) sit in LDS, lane-minor.
// Problem constants (Model, bounds) are uniform: read with scalar loads from a constant buffer.
//
// Riccati stage k in registers (closed forms of model.hpp, structure of G = [A~ B~] exploited):
//   ph = p + P c,  W_u = P B~  (one pass over the 153 packed P entries)
//   g = G^T ph + h,  Q_uu = B~^T W_u + H_uu,  Q_xu = A^T W_u + H_xu
//   Q_uu = L L^T (inertia test),  Z = L^-1 Q_ux,  K = -L^-T Z,  k = -Q_uu^-1 g_u
//   P_k = H_xx + A^T P_xx A - Z^T Z   (column groups of A sharing their sparsity, P re-read from HBM)
namespace lafse3 {
namespace lane {

constexpr int SXL = MAXN + 1;
// ---- per-lane workspace slots
constexpr int O_X = 0;                     // x[i][k]   13 x SXL
constexpr int O_U = O_X + NX * SXL;        // u[a][k]
constexpr int O_LAM = O_U + NU * SXL;      // lambda[i][k] (k < N)
constexpr int O_ZLU = O_LAM + NX * SXL;
constexpr int O_ZUU = O_ZLU + NU * SXL;
constexpr int O_ZLW = O_ZUU + NU * SXL;    // [c][k], k = 1..N
constexpr int O_ZUW = O_ZLW + 3 * SXL;
constexpr int O_DX = O_ZUW + 3 * SXL;      // Newton step
constexpr int O_DU = O_DX + NX * SXL;
constexpr int O_LP = O_DU + NU * SXL;      // lambda+ (full multiplier of the step)
constexpr int O_RQ = O_LP + NX * SXL;      // refinement right-hand side (x rows, u rows, dynamics rows)
constexpr int O_RR = O_RQ + NX * SXL;
constexpr int O_RC = O_RR + NU * SXL;
constexpr int O_EDX = O_RC + NX * SXL;     // refinement correction (kept for the revert)
constexpr int O_EDU = O_EDX + NX * SXL;
constexpr int O_ELP = O_EDU + NU * SXL;
constexpr int O_CC = O_ELP + NX * SXL;     // dynamics defect c_k of the last factorisation
constexpr int O_WK = O_CC + NX * SXL;      // traversal weight w_k
constexpr int O_PU = O_WK + SXL;           // u~ rows of P_{k+1}: P_xu~ [i][b] (52) | P_u~u~ packed (10)
constexpr int O_DD = O_PU + 64;            // refinement: forward-propagated dynamics defect d[i][k]
constexpr int O_K = O_DD + NX * SXL;       // [k][a][j] 4 x 17
constexpr int O_KK = O_K + MAXN * NU * NA; // [k][a]
constexpr int O_L = O_KK + MAXN * NU;      // [k][10]
constexpr int O_PN = O_L + MAXN * 10;      // terminal gradient p_N (13)
constexpr int O_PV = O_PN + 16;            // p_k carried between stages (17)
constexpr int O_FT = O_PV + 24;            // filter
constexpr int O_FP = O_FT + FMAX;
constexpr int O_CST = O_FP + FMAX;         // per-instance constants (C_* below)
constexpr int NSLOT = O_CST + 48;
constexpr int64_t BLOCK_DOUBLES = (int64_t)NSLOT * 64;

// ---- per-instance constants (slots O_CST + C_*)
constexpr int C_ST = 0, C_SG = 16, C_TRT = 32, C_TRG = 33, C_GOAL = 34, C_PTRA = 37, C_UL = 40, NCL = 44;

struct DevConst {
    Model M;
    double ulo, uhi, wlo, whi;          // bounds relaxed by bound_relax (IPOPT)
    double u_lb, u_ub, w_lb, w_ub;
    double tol, acceptable_tol, mu_init, tra_w_peak, tra_w_decay, wing_len, d_min;
    int N, max_iter, acceptable_iter, lsq_mult_init;
};

__host__ inline DevConst make_devconst(const lafse3_params &p)
{
    DevConst d;
    d.M = make_model(p);
    d.ulo = p.u_lb - p.bound_relax * fmax(1.0, fabs(p.u_lb));
    d.uhi = p.u_ub + p.bound_relax * fmax(1.0, fabs(p.u_ub));
    d.wlo = p.w_lb - p.bound_relax * fmax(1.0, fabs(p.w_lb));
    d.whi = p.w_ub + p.bound_relax * fmax(1.0, fabs(p.w_ub));
    d.u_lb = p.u_lb; d.u_ub = p.u_ub; d.w_lb = p.w_lb; d.w_ub = p.w_ub;
    d.tol = p.tol; d.acceptable_tol = p.acceptable_tol; d.mu_init = p.mu_init;
    d.tra_w_peak = p.tra_w_peak; d.tra_w_decay = p.tra_w_decay; d.wing_len = p.wing_len; d.d_min = p.d_min;
    d.N = p.horizon; d.max_iter = p.max_iter; d.acceptable_iter = p.acceptable_iter; d.lsq_mult_init = p.lsq_mult_init;
    return d;
}

typedef __attribute__((address_space(4))) const DevConst cDevConst;

// LDS: the x-x block of the Riccati cost-to-go P_{k+1} (packed upper 13x13, 91 doubles per lane,
// lane-minor so every ds_read_b64 of one entry by the wave is conflict-free).  46.6 KB per wave.
constexpr int NPX = NX * (NX + 1) / 2;
__shared__ double sP[NPX * 64];
__host__ __device__ constexpr int up13(int i, int j)
{
    return i <= j ? i * NX - i * (i - 1) / 2 + (j - i) : j * NX - j * (j - 1) / 2 + (i - j);
}
typedef __attribute__((address_space(3))) double ldouble;
__device__ inline double pl_ld(int i, int j) { return ((ldouble *)sP)[up13(i, j) * 64 + threadIdx.x]; }
__device__ inline void pl_st(int i, int j, double v) { ((ldouble *)sP)[up13(i, j) * 64 + threadIdx.x] = v; }
// Compiler memory barrier between phases: the accesses are per lane with compile-time offsets, so
// without it the optimiser would promote the whole LDS matrix into registers across the stage loop.
#define MEMBAR() asm volatile("" ::: "memory")
__shared__ unsigned long long *sPT;       // debug phase timers of this wave (nullable), see lafse3_debug_timers

// phase timers (s_memtime cycles, one accumulator set per wave, written by the first active lane, so a
// phase is counted whenever ANY lane of the wave runs it): 0 init, 1 errors, 3 backward, 4 forward,
// 5 adjoint, 6 residual, 7 refine-backward, 8 line search, 9 accept, 10 reward, 11 newton step (inclusive)
#define LT_BEGIN unsigned long long _lt0 = sPT ? __builtin_amdgcn_s_memtime() : 0ull
#define LT_COUNT(i)                                                                          \
    do {                                                                                     \
        if (sPT && threadIdx.x == __builtin_ctzll(__builtin_amdgcn_read_exec())) sPT[i] += 1; \
    } while (0)
#define LT_END(i)                                                           \
    do {                                                                    \
        if (sPT) {                                                          \
            const unsigned long long _lt1 = __builtin_amdgcn_s_memtime();   \
            if (threadIdx.x == __builtin_ctzll(__builtin_amdgcn_read_exec())) \
                sPT[i] += _lt1 - _lt0;                                      \
            _lt0 = _lt1;                                                    \
        }                                                                   \
    } while (0)

// Scheduling fence: keeps the machine scheduler from hoisting a whole pass worth of independent loads
// above the arithmetic that consumes them (which would need more registers than exist and spill).
#define FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ inline uint64_t rfl64(uint64_t v)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// One lane's view of its instance's slots: uniform block base + slot offset computed on the scalar
// unit (the slot depends only on loop counters, identical across the active lanes), plus one 32-bit
// lane offset.  Plain global loads/stores, so the scheduler can batch independent loads.
typedef __attribute__((address_space(1))) char gchar;

struct LB {
    uint64_t base;    // uniform
    uint32_t off;     // lane * 8
    __device__ inline gdouble *ptr(int slot) const
    {
        const uint64_t b = base + (uint64_t)((uint32_t)slot * 512u);
        return (gdouble *)((gchar *)b + off);
    }
    __device__ inline double ld(int slot) const { return *ptr(slot); }
    __device__ inline void st(int slot, double x) const { *ptr(slot) = x; }
    // per-lane (divergent) slot index
    __device__ inline double ld_div(int slot) const { return *(gdouble *)((gchar *)base + (off + (uint32_t)slot * 512u)); }
    __device__ inline void st_div(int slot, double x) const { *(gdouble *)((gchar *)base + (off + (uint32_t)slot * 512u)) = x; }
    struct Ref {
        const LB *w;
        int slot;
        __device__ inline operator double() const { return w->ld(slot); }
        __device__ inline Ref &operator=(double x) { w->st(slot, x); return *this; }
        __device__ inline Ref &operator=(const Ref &o) { w->st(slot, (double)o); return *this; }
    };
    __device__ inline Ref operator[](int slot) const { return Ref{this, slot}; }
};

__device__ inline LB make_lb(double *ws_block)
{
    LB W;
    W.base = rfl64((uint64_t)ws_block);
    W.off = threadIdx.x * 8u;
    return W;
}

__device__ inline const cDevConst &dconst(const DevConst *p) { return *(const cDevConst *)rfl64((uint64_t)p); }

__device__ inline double cst(const LB &W, int e) { return W[O_CST + e]; }
__host__ __device__ constexpr int up4(int a, int b) { return a <= b ? a * 4 - a * (a - 1) / 2 + (b - a) : b * 4 - b * (b - 1) / 2 + (a - b); }
__host__ __device__ constexpr int pu_xu(int i, int b) { return O_PU + i * NU + b; }
__host__ __device__ constexpr int pu_uu(int a, int b) { return O_PU + NX * NU + up4(a, b); }

// uniform Model from the constant buffer (scalar loads; Model is a plain struct of doubles).
// The lane variant is specialised for the reference's zero goal-attitude weight (quad_policy.py:38
// wqf=0): the host routes wqf != 0 to the wave variant, so the Sg terms fold away here.
__device__ inline Model load_model(const cDevConst &D)
{
    static_assert(sizeof(Model) % sizeof(double) == 0, "Model must be all doubles");
    typedef __attribute__((address_space(4))) const double cdouble;
    Model m;
    double *d = reinterpret_cast<double *>(&m);
    cdouble *src = reinterpret_cast<cdouble *>(&D.M);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(Model) / sizeof(double)); ++i) d[i] = src[i];
    m.wqf = 0.0;
    return m;
}

struct Inst {      // per-lane constants pulled from LDS
    double goal[3], ptra[3];
};

__device__ inline void load_att(const LB &W, const Model &M, Attitude &at)
{
#pragma unroll
    for (int i = 0; i < 16; ++i) at.St[i] = cst(W, C_ST + i);
#pragma unroll
    for (int i = 0; i < 16; ++i) at.Sg[i] = 0.0;      // unused: wqf == 0 (see load_model)
    at.trRt = cst(W, C_TRT);
    at.trRg = 3.0;
}
__device__ inline void load_inst(const LB &W, Inst &I)
{
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        I.goal[i] = cst(W, C_GOAL + i);
        I.ptra[i] = cst(W, C_PTRA + i);
    }
}

__device__ inline void ldv(const LB &W, int base, int k, int n, double *v)
{
#pragma unroll
    for (int i = 0; i < n; ++i) v[i] = W[base + i * SXL + k];
}
__device__ inline void stv(const LB &W, int base, int k, int n, const double *v)
{
#pragma unroll
    for (int i = 0; i < n; ++i) W[base + i * SXL + k] = v[i];
}
__device__ inline void ld_uprev(const LB &W, int k, double *up)
{
    if (k == 0) {
#pragma unroll
        for (int a = 0; a < NU; ++a) up[a] = cst(W, C_UL + a);
    } else {
        ldv(W, O_U, k - 1, NU, up);
    }
}

// s * gradient of (w_k tra + path) at x (k = 1..N; w_N = 0: final cost)
__device__ inline void grad_xs(const Model &M, const Attitude &at, const Inst &I, double wk, double s, const double *x,
                               double *g)
{
    state_cost_grad(M, at, I.goal, I.ptra, wk, x, g);
#pragma unroll
    for (int i = 0; i < NX; ++i) g[i] *= s;
}

// s * gradient w.r.t. u_k
__device__ inline void grad_us(const Model &M, double s, int k, int N, const double *uk, const double *up,
                               const double *un, double *g)
{
#pragma unroll
    for (int a = 0; a < NU; ++a) {
        double v = 2 * M.wthrust * uk[a] + M.du_w * 2 * (uk[a] - up[a]);
        if (k + 1 < N) v += -M.du_w * 2 * (un[a] - uk[a]);
        g[a] = v * s;
    }
}

__device__ inline void bar(double v, double lo, double hi, double zl, double zu, double mu, double &g, double &sg)
{
    const double isl = 1.0 / (v - lo), isu = 1.0 / (hi - v);
    g = -mu * isl + mu * isu;
    sg = zl * isl + zu * isu;
}

// diagonal of the terminal cost-to-go P_N (final cost Hessian + omega barrier + delta_w; wqf == 0)
__device__ inline void pn_diag(const cDevConst &D, const Model &M, const LB &W, int N, double s, double mu, double dw,
                               int lsq, double *pd)
{
#pragma unroll
    for (int i = 0; i < NX; ++i) {
        double v;
        if (lsq) {
            v = 1.0;
        } else {
            v = (i < 3) ? s * 2 * M.wrf : (i < 6) ? s * 2 * M.wvf : (i >= 10) ? s * 2 * M.wwf : 0.0;
            v += dw;
        }
        pd[i] = v;
    }
    if (!lsq)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double gb, sg;
            bar(W[O_X + (10 + c) * SXL + N], D.wlo, D.whi, W[O_ZLW + c * SXL + N], W[O_ZUW + c * SXL + N], mu, gb, sg);
            pd[10 + c] += sg;
        }
}

// forward / backward halves of the packed 4x4 Cholesky solve (L = l00 l10 l11 l20 l21 l22 l30 l31 l32 l33);
// the diagonal is used through its reciprocals iL (4 divisions per stage instead of 8 per right-hand side)
__device__ inline void chol_inv_diag(const double *L, double *iL)
{
    iL[0] = 1.0 / L[0]; iL[1] = 1.0 / L[2]; iL[2] = 1.0 / L[5]; iL[3] = 1.0 / L[9];
}
__device__ inline void chol_fwd(const double *L, const double *iL, double &b0, double &b1, double &b2, double &b3)
{
    b0 = b0 * iL[0];
    b1 = (b1 - L[1] * b0) * iL[1];
    b2 = (b2 - L[3] * b0 - L[4] * b1) * iL[2];
    b3 = (b3 - L[6] * b0 - L[7] * b1 - L[8] * b2) * iL[3];
}
__device__ inline void chol_bwd(const double *L, const double *iL, double &b0, double &b1, double &b2, double &b3)
{
    b3 = b3 * iL[3];
    b2 = (b2 - L[8] * b3) * iL[2];
    b1 = (b1 - L[4] * b2 - L[7] * b3) * iL[1];
    b0 = (b0 - L[1] * b1 - L[3] * b2 - L[6] * b3) * iL[0];
}

// B~[l][a] (rows of [B; I]): structural zeros are compile-time after unrolling
__device__ inline double bt_coef(const Model &M, const double *bv, int l, int a)
{
    if (l >= 3 && l < 6) return bv[l - 3];
    if (l >= 10 && l < 13) return Bw(M, l - 10, a);
    if (l >= 13) return (l - 13 == a) ? 1.0 : 0.0;
    return 0.0;
}
__device__ inline bool bt_nz(int l, int a)
{
    if (l >= 3 && l < 6) return true;
    if (l == 10) return a == 1 || a == 3;
    if (l == 11) return a == 0 || a == 2;
    if (l == 12) return true;
    if (l >= 13) return l - 13 == a;
    return false;
}

// ------------------------------------------------------------------------------------------------
// KKT errors (oracle compute_errors order: u rows over k, then x rows over k = 1..N)
struct Errs {
    double dinf, pinf, cmu, c0, sd, sc;
};

__device__ __forceinline__ Errs lk_errors(const DevConst *dcp, double *wsb, double s, double mu)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    Attitude at;
    load_att(W, M, at);
    Inst I;
    load_inst(W, I);
    double dinf = 0, pinf = 0, cmu = 0, c0 = 0, smult = 0, sz = 0;
    double up[NU], uk[NU], un[NU], xk[NX];
    ld_uprev(W, 0, up);
    ldv(W, O_U, 0, NU, uk);
    ldv(W, O_X, 0, NX, xk);
    for (int k = 0; k < N; ++k) {
        if (k + 1 < N) ldv(W, O_U, k + 1, NU, un);
        double lk[NX], x1[NX];
        ldv(W, O_LAM, k, NX, lk);
        ldv(W, O_X, k + 1, NX, x1);
        double gu[NU], btl[NU];
        grad_us(M, s, k, N, uk, up, un, gu);
        Bt_times(M, xk, lk, btl);
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            const double zl = W[O_ZLU + a * SXL + k], zu = W[O_ZUU + a * SXL + k];
            const double acc = gu[a] + btl[a] - zl + zu;
            dinf = fmax(dinf, fabs(acc));
            const double sl = uk[a] - D.ulo, su = D.uhi - uk[a];
            cmu = fmax(cmu, fmax(fabs(sl * zl - mu), fabs(su * zu - mu)));
            c0 = fmax(c0, fmax(fabs(sl * zl), fabs(su * zu)));
            sz += zl + zu;
        }
        double xn[NX];
        f_disc(M, xk, uk, xn);
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            pinf = fmax(pinf, fabs(xn[i] - x1[i]));
            smult += fabs(lk[i]);
        }
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            up[a] = uk[a];
            uk[a] = un[a];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) xk[i] = x1[i];
    }
    for (int k = 1; k <= N; ++k) {
        double x1[NX], g[NX], lp[NX];
        ldv(W, O_X, k, NX, x1);
        ldv(W, O_LAM, k - 1, NX, lp);
        grad_xs(M, at, I, (k < N) ? (double)W[O_WK + k] : 0.0, s, x1, g);
#pragma unroll
        for (int i = 0; i < NX; ++i) g[i] -= lp[i];
        if (k < N) {
            double u1[NU], l1[NX], atl[NX];
            ldv(W, O_U, k, NU, u1);
            ldv(W, O_LAM, k, NX, l1);
            At_times(M, x1, u1, l1, atl);
#pragma unroll
            for (int i = 0; i < NX; ++i) g[i] += atl[i];
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double zl = W[O_ZLW + c * SXL + k], zu = W[O_ZUW + c * SXL + k];
            g[10 + c] += -zl + zu;
            const double sl = x1[10 + c] - D.wlo, su = D.whi - x1[10 + c];
            cmu = fmax(cmu, fmax(fabs(sl * zl - mu), fabs(su * zu - mu)));
            c0 = fmax(c0, fmax(fabs(sl * zl), fabs(su * zu)));
            sz += zl + zu;
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) dinf = fmax(dinf, fabs(g[i]));
    }
    const double smax = 100.0;
    const double n_mult = (double)(N * NX) + (double)(N * NU * 2 + N * 3 * 2);
    const double n_z = (double)(N * NU * 2 + N * 3 * 2);
    Errs E;
    E.sd = fmax(smax, (smult + sz) / n_mult) / smax;
    E.sc = fmax(smax, sz / n_z) / smax;
    E.dinf = dinf;
    E.pinf = pinf;
    E.cmu = cmu;
    E.c0 = c0;
    return E;
}

__device__ inline double err_val(const Errs &E, int with_mu)
{
    const double c = with_mu ? E.cmu : E.c0;
    return fmax(E.dinf / E.sd, fmax(E.pinf, c / E.sc));
}

// objective J at (x + alpha dx, u + alpha du) (oracle objective_J order)
__device__ inline double stage_J(const Model &M, const Attitude &at, const Inst &I, double wk, const double *xk,
                                 const double *uk, const double *up)
{
    double c = state_cost(M, at, I.goal, I.ptra, wk, xk);
    double th = 0, sm = 0;
#pragma unroll
    for (int a = 0; a < NU; ++a) {
        th += uk[a] * uk[a];
        sm += (uk[a] - up[a]) * (uk[a] - up[a]);
    }
    return c + M.wthrust * th + M.du_w * sm;
}

struct Merit {
    double theta, phi;
    int ok;
};

// theta = ||c||_1 and barrier objective phi at step length alpha (oracle eval_merit order)
__device__ __forceinline__ Merit lk_merit(const DevConst *dcp, double *wsb, double s, double mu, double alpha)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    Attitude at;
    load_att(W, M, at);
    Inst I;
    load_inst(W, I);
    double th = 0, lb = 0, J = 0;
    int good = 1;
    double xk[NX], up[NU];
    ld_uprev(W, 0, up);
#pragma unroll
    for (int i = 0; i < NX; ++i) xk[i] = W[O_X + i * SXL] + alpha * W[O_DX + i * SXL];
    for (int k = 0; k < N; ++k) {
        double x1[NX], uk[NU], xn[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) x1[i] = W[O_X + i * SXL + k + 1] + alpha * W[O_DX + i * SXL + k + 1];
#pragma unroll
        for (int a = 0; a < NU; ++a) uk[a] = W[O_U + a * SXL + k] + alpha * W[O_DU + a * SXL + k];
        f_disc(M, xk, uk, xn);
#pragma unroll
        for (int i = 0; i < NX; ++i) th += fabs(xn[i] - x1[i]);
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            const double sl = uk[a] - D.ulo, su = D.uhi - uk[a];
            if (!(sl > 0) || !(su > 0)) good = 0;
            lb += log(sl) + log(su);
        }
        J += stage_J(M, at, I, W[O_WK + k], xk, uk, up);
#pragma unroll
        for (int i = 0; i < NX; ++i) xk[i] = x1[i];
#pragma unroll
        for (int a = 0; a < NU; ++a) up[a] = uk[a];
    }
    J += state_cost(M, at, I.goal, I.ptra, 0.0, xk);
    for (int k = 1; k <= N; ++k) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double v = W[O_X + (10 + c) * SXL + k] + alpha * W[O_DX + (10 + c) * SXL + k];
            const double sl = v - D.wlo, su = D.whi - v;
            if (!(sl > 0) || !(su > 0)) good = 0;
            lb += log(sl) + log(su);
        }
    }
    Merit R;
    R.theta = th;
    R.phi = s * J - mu * lb;
    R.ok = good && isfinite(R.phi) && isfinite(th);
    return R;
}

__device__ __forceinline__ double lk_objective(const DevConst *dcp, double *wsb)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    Attitude at;
    load_att(W, M, at);
    Inst I;
    load_inst(W, I);
    double J = 0, up[NU];
    ld_uprev(W, 0, up);
    for (int k = 0; k < N; ++k) {
        double xk[NX], uk[NU];
        ldv(W, O_X, k, NX, xk);
        ldv(W, O_U, k, NU, uk);
        J += stage_J(M, at, I, W[O_WK + k], xk, uk, up);
#pragma unroll
        for (int a = 0; a < NU; ++a) up[a] = uk[a];
    }
    double xN[NX];
    ldv(W, O_X, N, NX, xN);
    return J + state_cost(M, at, I.goal, I.ptra, 0.0, xN);
}

// ------------------------------------------------------------------------------------------------
// Riccati factorisation sweep.  Returns 1 on success, 0 when some Q_uu is not positive definite.
//
// P_{k+1} lives split: its x-x block in LDS (sP, updated in place stage after stage), its u~ rows in the
// lane's HBM slots (Pst[k], also the full copy the refinement sweeps re-read).  Global loads of a stage
// are issued before its global stores where possible (gfx9 counts both on vmcnt, so a load issued after
// a store waits for that store).
//
// A^T P A in place: A = (I + E_w)(I + E_q)(I + E_v) exactly (the cross products of the column groups'
// E vanish), so P <- A_w^T P A_w, then A_q, then A_v; each factor rewrites only its own rows/columns
// and needs a register buffer of one column group (<= 4 x 13).

struct ACols {
    double q[4], w[3], Tm, dt, hdt, ax, ay, az;
};

// group w: E[q_b][w_c] = dt/2 Xi(q)[b][c], E[w_d][w_c] = dt Jw[d][c]
__device__ inline void congr_w(const ACols &a)
{
    const double *q = a.q, *w = a.w;
    const double Xi[4][3] = {{-q[1], -q[2], -q[3]}, {q[0], -q[3], q[2]}, {q[3], q[0], -q[1]}, {-q[2], q[1], q[0]}};
    const double Jw[3][3] = {{0.0, -a.ax * w[2], -a.ax * w[1]},
                             {-a.ay * w[2], 0.0, -a.ay * w[0]},
                             {-a.az * w[1], -a.az * w[0], 0.0}};
    double Eq[4][3], Ew[3][3];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int c = 0; c < 3; ++c) Eq[b][c] = a.hdt * Xi[b][c];
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int c = 0; c < 3; ++c) Ew[d][c] = a.dt * Jw[d][c];
    double C[NX][3];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double acc = pl_ld(m, 10 + c);
#pragma unroll
            for (int b = 0; b < 4; ++b) acc += pl_ld(m, 6 + b) * Eq[b][c];
#pragma unroll
            for (int d = 0; d < 3; ++d)
                if (d != c) acc += pl_ld(m, 10 + d) * Ew[d][c];
            C[m][c] = acc;
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
        for (int m = 0; m < 10; ++m) pl_st(m, 10 + c, C[m][c]);
#pragma unroll
        for (int e = 0; e <= c; ++e) {
            double acc = C[10 + e][c];
#pragma unroll
            for (int b = 0; b < 4; ++b) acc += Eq[b][e] * C[6 + b][c];
#pragma unroll
            for (int d = 0; d < 3; ++d)
                if (d != e) acc += Ew[d][e] * C[10 + d][c];
            pl_st(10 + e, 10 + c, acc);
        }
    }
}

// group q: E[v_i][q_c] = dt Tm dg/dq (Dg[i][c]), E[q_b][q_c] = dt/2 Omega(w)[b][c]
__device__ inline void congr_q(const ACols &a)
{
    const double *q = a.q, *w = a.w;
    const double dtt = a.dt * a.Tm;
    const double Ev[3][4] = {{dtt * 2 * q[2], dtt * 2 * q[3], dtt * 2 * q[0], dtt * 2 * q[1]},
                             {-dtt * 2 * q[1], -dtt * 2 * q[0], dtt * 2 * q[3], dtt * 2 * q[2]},
                             {0.0, -dtt * 4 * q[1], -dtt * 4 * q[2], 0.0}};
    const double Om[4][4] = {{0.0, -w[0], -w[1], -w[2]},
                             {w[0], 0.0, w[2], -w[1]},
                             {w[1], -w[2], 0.0, w[0]},
                             {w[2], w[1], -w[0], 0.0}};
    double Eq[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int c = 0; c < 4; ++c) Eq[b][c] = a.hdt * Om[b][c];
    double C[NX][4];
#pragma unroll
    for (int m = 0; m < NX; ++m) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            double acc = pl_ld(m, 6 + c);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (!(i == 2 && (c == 0 || c == 3))) acc += pl_ld(m, 3 + i) * Ev[i][c];
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (b != c) acc += pl_ld(m, 6 + b) * Eq[b][c];
            C[m][c] = acc;
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int m = 0; m < NX; ++m)
            if (m < 6 || m >= 10) pl_st(m, 6 + c, C[m][c]);
#pragma unroll
        for (int e = 0; e <= c; ++e) {
            double acc = C[6 + e][c];
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (!(i == 2 && (e == 0 || e == 3))) acc += Ev[i][e] * C[3 + i][c];
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (b != e) acc += Eq[b][e] * C[6 + b][c];
            pl_st(6 + e, 6 + c, acc);
        }
    }
}

// group v: E[r_a][v_a] = dt
__device__ inline void congr_v(const ACols &a)
{
    double C[NX][3];
#pragma unroll
    for (int m = 0; m < NX; ++m)
#pragma unroll
        for (int c = 0; c < 3; ++c) C[m][c] = pl_ld(m, 3 + c) + a.dt * pl_ld(m, c);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
        for (int m = 0; m < NX; ++m)
            if (m < 3 || m >= 6) pl_st(m, 3 + c, C[m][c]);
#pragma unroll
        for (int e = 0; e <= c; ++e) pl_st(3 + e, 3 + c, C[3 + e][c] + a.dt * C[e][c]);
    }
}

__device__ __forceinline__ int lk_backward(const DevConst *dcp, double *wsb, double s, double mu, double dw, int lsq)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    const double dt = M.dt;
    const double d2 = 2 * M.du_w * s;           // |u - u_prev|^2 Hessian scale
    const double hu_ = lsq ? 0.0 : d2;          // u~ blocks of H~ (zero in the least-squares system)
    // ---- terminal P_N, p_N
    {
        Attitude at;
        load_att(W, M, at);
        Inst I;
        load_inst(W, I);
        double xN[NX], g[NX], sgw[3] = {0, 0, 0};
        ldv(W, O_X, N, NX, xN);
        double zl[3], zu[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            zl[c] = W[O_ZLW + c * SXL + N];
            zu[c] = W[O_ZUW + c * SXL + N];
        }
        grad_xs(M, at, I, 0.0, s, xN, g);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if (lsq) {
                g[10 + c] += -zl[c] + zu[c];
            } else {
                double gb, sg;
                bar(xN[10 + c], D.wlo, D.whi, zl[c], zu[c], mu, gb, sg);
                g[10 + c] += gb;
                sgw[c] = sg;
            }
        }
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int j = i; j < NX; ++j) {
                double v = 0.0;
                if (i == j) {
                    if (lsq) {
                        v = 1.0;
                    } else {
                        v = (i < 3) ? s * 2 * M.wrf : (i < 6) ? s * 2 * M.wvf : (i >= 10) ? s * 2 * M.wwf : 0.0;
                        v += dw;
                        if (i >= 10) v += sgw[i - 10];
                    }
                }
                pl_st(i, j, v);
            }
#pragma unroll
        for (int e = 0; e < 64; ++e) W[O_PU + e] = 0.0;
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            W[O_PN + i] = g[i];
            W[O_PV + i] = g[i];
        }
#pragma unroll
        for (int a = 0; a < NU; ++a) W[O_PV + NX + a] = 0.0;
    }
    MEMBAR();
    for (int k = N - 1; k >= 0; --k) {
        ACols ac;
        double gx[NX], gu[NU], hut[NU], Ruu[NU], qu[4], c[NX];
        // ---- phase 1: stage data, ph = p + P c~, g = G^T ph + h
        {
            double xk[NX], uk[NU], up[NU], hu[NU], ph[NA], zlu[NU], zuu[NU], pxu[NX][NU];
            ldv(W, O_X, k, NX, xk);
            ldv(W, O_U, k, NU, uk);
            ld_uprev(W, k, up);
#pragma unroll
            for (int i = 0; i < NA; ++i) ph[i] = W[O_PV + i];
#pragma unroll
            for (int a = 0; a < NU; ++a) {
                zlu[a] = W[O_ZLU + a * SXL + k];
                zuu[a] = W[O_ZUU + a * SXL + k];
            }
            if (lsq) {
#pragma unroll
                for (int i = 0; i < NX; ++i) c[i] = 0.0;
            } else {
                double xn[NX], x1[NX];
                ldv(W, O_X, k + 1, NX, x1);
                f_disc(M, xk, uk, xn);
#pragma unroll
                for (int i = 0; i < NX; ++i) c[i] = xn[i] - x1[i];
            }
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int b = 0; b < NU; ++b) pxu[i][b] = W[pu_xu(i, b)];
#pragma unroll
            for (int i = 0; i < 4; ++i) ac.q[i] = xk[6 + i];
#pragma unroll
            for (int i = 0; i < 3; ++i) ac.w[i] = xk[10 + i];
            ac.Tm = (uk[0] + uk[1] + uk[2] + uk[3]) * M.imass;
            ac.dt = dt; ac.hdt = 0.5 * dt; ac.ax = M.ax; ac.ay = M.ay; ac.az = M.az;
#pragma unroll
            for (int a = 0; a < NU; ++a) {
                double r = s * (2 * M.wthrust * uk[a] + 2 * M.du_w * (uk[a] - up[a]));
                if (lsq) {
                    r += -zlu[a] + zuu[a];
                    Ruu[a] = 1.0;
                } else {
                    double gb, sg;
                    bar(uk[a], D.ulo, D.uhi, zlu[a], zuu[a], mu, gb, sg);
                    r += gb;
                    Ruu[a] = s * (2 * M.wthrust + 2 * M.du_w) + sg;
                }
                hu[a] = r;
                hut[a] = -d2 * (uk[a] - up[a]);
            }
            // ph_x += P_xx c (LDS), ph_u~ += P_u~x c
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double acc = ph[i];
#pragma unroll
                for (int j = 0; j < NX; ++j) acc += pl_ld(i, j) * c[j];
                ph[i] = acc;
            }
#pragma unroll
            for (int b = 0; b < NU; ++b)
#pragma unroll
                for (int j = 0; j < NX; ++j) ph[NX + b] += pxu[j][b] * c[j];
            At_times(M, xk, uk, ph, gx);
            double bt[NU];
            Bt_times(M, xk, ph, bt);
#pragma unroll
            for (int a = 0; a < NU; ++a) gu[a] = bt[a] + ph[NX + a] + hu[a];
            qu[0] = qu[1] = qu[2] = qu[3] = 0.0;
            if (k >= 1) {
                Attitude at;
                load_att(W, M, at);
                Inst I;
                load_inst(W, I);
                double hx[NX], zl[3], zu[3];
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    zl[cc] = W[O_ZLW + cc * SXL + k];
                    zu[cc] = W[O_ZUW + cc * SXL + k];
                }
                const double wk = W[O_WK + k];
                grad_xs(M, at, I, wk, s, xk, hx);
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    if (lsq) {
                        hx[10 + cc] += -zl[cc] + zu[cc];
                    } else {
                        double gb, sg;
                        bar(xk[10 + cc], D.wlo, D.whi, zl[cc], zu[cc], mu, gb, sg);
                        hx[10 + cc] += gb;
                    }
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) gx[i] += hx[i];
                if (!lsq) {
                    const double *q = ac.q;
                    const double a0 = W[O_LAM + 3 * SXL + k], a1 = W[O_LAM + 4 * SXL + k], a2 = W[O_LAM + 5 * SXL + k];
                    qu[0] = M.dtm * (2 * a0 * q[2] - 2 * a1 * q[1]);
                    qu[1] = M.dtm * (2 * a0 * q[3] - 2 * a1 * q[0] - 4 * a2 * q[1]);
                    qu[2] = M.dtm * (2 * a0 * q[0] + 2 * a1 * q[3] - 4 * a2 * q[2]);
                    qu[3] = M.dtm * (2 * a0 * q[1] + 2 * a1 * q[2]);
                }
            }
        }
        // ---- phase 2: W_u = P B~ ; Q_uu = B~^T W_u + R, Q_xu = A^T W_u[x rows] + H_xu
        double Quu[NU][NU], Qxu[NX][NU];
        {
            const double *q = ac.q;
            const double g0 = 2 * (q[1] * q[3] + q[0] * q[2]);
            const double g1 = 2 * (q[2] * q[3] - q[0] * q[1]);
            const double g2 = 1 - 2 * (q[1] * q[1] + q[2] * q[2]);
            const double bv[3] = {M.dtm * g0, M.dtm * g1, M.dtm * g2};
            double xq[NX], uq[NU];
#pragma unroll
            for (int i = 0; i < NX; ++i) xq[i] = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i) xq[6 + i] = q[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) xq[10 + i] = ac.w[i];
            uq[0] = ac.Tm * M.mass; uq[1] = uq[2] = uq[3] = 0.0;
            // u~ rows: wt[b][a] = P_u~x B[:, a] + P_u~u~[b][a]
            double wt[NU][NU];
            {
                double pxu[NX][NU];
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int b = 0; b < NU; ++b) pxu[i][b] = W[pu_xu(i, b)];
#pragma unroll
                for (int b = 0; b < NU; ++b)
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        double acc = W[pu_uu(b, a)];
#pragma unroll
                        for (int l = 0; l < NX; ++l)
                            if (bt_nz(l, a)) acc += pxu[l][b] * bt_coef(M, bv, l, a);
                        wt[b][a] = acc;
                    }
                // x rows, one column at a time
#pragma unroll
                for (int b = 0; b < NU; ++b) {
                    double col[NX], bt[NU], at_[NX];
#pragma unroll
                    for (int i = 0; i < NX; ++i) {
                        double acc = pxu[i][b];
#pragma unroll
                        for (int l = 0; l < NX; ++l)
                            if (bt_nz(l, b)) acc += pl_ld(i, l) * bt_coef(M, bv, l, b);
                        col[i] = acc;
                    }
                    Bt_times(M, xq, col, bt);
                    At_times(M, xq, uq, col, at_);
#pragma unroll
                    for (int a = 0; a <= b; ++a) Quu[a][b] = bt[a] + wt[a][b];
                    Quu[b][b] += Ruu[b] + dw;
#pragma unroll
                    for (int i = 0; i < NX; ++i) Qxu[i][b] = at_[i];
#pragma unroll
                    for (int r = 0; r < 4; ++r) Qxu[6 + r][b] += qu[r];
                }
            }
        }
        // ---- phase 3: Cholesky of Q_uu (same order as chol4 in the oracle / wave kernel)
        double L[10], iL[4];
        int ok = 1;
        {
            double d = Quu[0][0];
            if (!(d > 0.0)) ok = 0;
            L[0] = sqrt(fmax(d, 1e-300));
            iL[0] = 1.0 / L[0];
            L[1] = Quu[0][1] * iL[0];
            L[3] = Quu[0][2] * iL[0];
            L[6] = Quu[0][3] * iL[0];
            d = Quu[1][1] - L[1] * L[1];
            if (!(d > 0.0)) ok = 0;
            L[2] = sqrt(fmax(d, 1e-300));
            iL[1] = 1.0 / L[2];
            L[4] = (Quu[1][2] - L[3] * L[1]) * iL[1];
            L[7] = (Quu[1][3] - L[6] * L[1]) * iL[1];
            d = Quu[2][2] - L[3] * L[3] - L[4] * L[4];
            if (!(d > 0.0)) ok = 0;
            L[5] = sqrt(fmax(d, 1e-300));
            iL[2] = 1.0 / L[5];
            L[8] = (Quu[2][3] - L[6] * L[3] - L[7] * L[4]) * iL[2];
            d = Quu[3][3] - L[6] * L[6] - L[7] * L[7] - L[8] * L[8];
            if (!(d > 0.0)) ok = 0;
            L[9] = sqrt(fmax(d, 1e-300));
            iL[3] = 1.0 / L[9];
        }
        if (!ok) return 0;
        // ---- phase 4: Z = L^-1 Q_ux (in place of Q_xu), gains K = -L^-T Z, k = -Q_uu^-1 g_u  (stores begin)
        stv(W, O_CC, k, NX, c);
#pragma unroll
        for (int e = 0; e < 10; ++e) W[O_L + k * 10 + e] = L[e];
        const int kb = O_K + k * NU * NA;
#pragma unroll
        for (int j = 0; j < NX; ++j) {
            double b0 = Qxu[j][0], b1 = Qxu[j][1], b2 = Qxu[j][2], b3 = Qxu[j][3];
            chol_fwd(L, iL, b0, b1, b2, b3);
            Qxu[j][0] = b0; Qxu[j][1] = b1; Qxu[j][2] = b2; Qxu[j][3] = b3;
            chol_bwd(L, iL, b0, b1, b2, b3);
            W[kb + 0 * NA + j] = -b0; W[kb + 1 * NA + j] = -b1; W[kb + 2 * NA + j] = -b2; W[kb + 3 * NA + j] = -b3;
        }
        double Zt[NU][NU];
#pragma unroll
        for (int b = 0; b < NU; ++b) {
            double e[4] = {0, 0, 0, 0};
            e[b] = -hu_;
            chol_fwd(L, iL, e[0], e[1], e[2], e[3]);
#pragma unroll
            for (int a = 0; a < NU; ++a) Zt[a][b] = e[a];
            chol_bwd(L, iL, e[0], e[1], e[2], e[3]);
#pragma unroll
            for (int a = 0; a < NU; ++a) W[kb + a * NA + NX + b] = -e[a];
        }
        double y0 = gu[0], y1 = gu[1], y2 = gu[2], y3 = gu[3];
        chol_fwd(L, iL, y0, y1, y2, y3);
        {
            double k0 = y0, k1 = y1, k2 = y2, k3 = y3;
            chol_bwd(L, iL, k0, k1, k2, k3);
            W[O_KK + k * NU + 0] = -k0; W[O_KK + k * NU + 1] = -k1;
            W[O_KK + k * NU + 2] = -k2; W[O_KK + k * NU + 3] = -k3;
        }
        if (k == 0) break;
        auto Z = [&](int a, int i) -> double { return Qxu[i][a]; };
        // ---- p_k = g + Q_x~u k  (= g - [Z Zt]^T y)
        const double yv[4] = {y0, y1, y2, y3};
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            double acc = gx[i];
#pragma unroll
            for (int a = 0; a < NU; ++a) acc -= Z(a, i) * yv[a];
            W[O_PV + i] = acc;
        }
#pragma unroll
        for (int b = 0; b < NU; ++b) {
            double acc = hut[b];
#pragma unroll
            for (int a = 0; a < NU; ++a) acc -= Zt[a][b] * yv[a];
            W[O_PV + NX + b] = acc;
        }
        // ---- phase 5: P_k u~ rows -> HBM (read back by the next stage's phases 1-2)
#pragma unroll
        for (int i = 0; i < NX; ++i)
#pragma unroll
            for (int b = 0; b < NU; ++b) {
                double acc = 0.0;
#pragma unroll
                for (int a = 0; a < NU; ++a) acc -= Z(a, i) * Zt[a][b];
                W[pu_xu(i, b)] = acc;
            }
#pragma unroll
        for (int a2 = 0; a2 < NU; ++a2)
#pragma unroll
            for (int b = a2; b < NU; ++b) {
                double acc = (a2 == b) ? hu_ : 0.0;
#pragma unroll
                for (int a = 0; a < NU; ++a) acc -= Zt[a][a2] * Zt[a][b];
                W[pu_uu(a2, b)] = acc;
            }
        // ---- phase 6: LDS P_xx <- A^T P_xx A in place
        MEMBAR();
        congr_w(ac);
        MEMBAR();
        congr_q(ac);
        MEMBAR();
        congr_v(ac);
        MEMBAR();
        // ---- phase 7: + H_xx - Z^T Z on LDS
        {
            double xk[NX], uk[NU], lk[NX];
            ldv(W, O_X, k, NX, xk);
            ldv(W, O_U, k, NU, uk);
            double sgw[3] = {0, 0, 0};
            StageHess H;
            if (lsq) {
                H.hr = H.hv = H.hw = 1.0;
#pragma unroll
                for (int e = 0; e < 16; ++e) H.qq[e] = ((e % 5) == 0) ? 1.0 : 0.0;
#pragma unroll
                for (int e = 0; e < 12; ++e) H.qw[e] = 0.0;
                H.wyz = H.wxz = H.wxy = 0.0;
            } else {
                ldv(W, O_LAM, k, NX, lk);
                double zl[3], zu[3];
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    zl[cc] = W[O_ZLW + cc * SXL + k];
                    zu[cc] = W[O_ZUW + cc * SXL + k];
                }
                const double wk = W[O_WK + k];
                Attitude at;
                load_att(W, M, at);
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) {
                    double gb;
                    bar(xk[10 + cc], D.wlo, D.whi, zl[cc], zu[cc], mu, gb, sgw[cc]);
                }
                stage_hessian(M, at, s, wk, xk, uk, lk, H);
            }
            auto hxx = [&](int i, int j) -> double {
                if (i == j) {
                    if (i < 3) return H.hr + dw;
                    if (i < 6) return H.hv + dw;
                    if (i < 10) return H.qq[(i - 6) * 5] + dw;
                    return H.hw + sgw[i - 10] + dw;
                }
                if (i >= 6 && i < 10 && j >= 6 && j < 10) return H.qq[(i - 6) * 4 + (j - 6)];
                if (i >= 6 && i < 10 && j >= 10) return H.qw[(i - 6) * 3 + (j - 10)];
                if (i == 10 && j == 11) return H.wxy;
                if (i == 10 && j == 12) return H.wxz;
                if (i == 11 && j == 12) return H.wyz;
                return 0.0;
            };
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int j = i; j < NX; ++j) {
                    double acc = pl_ld(i, j) + hxx(i, j);
#pragma unroll
                    for (int a = 0; a < NU; ++a) acc -= Z(a, i) * Z(a, j);
                    pl_st(i, j, acc);
                }
        }
        MEMBAR();
    }
    return 1;
}

// ---- forward rollout of the step: du = K dx~ + k,  dx_{k+1} = A dx + B du + c
// refine: the system is the defect-shifted one (c = 0, x = x^ + d, see lk_backward_refine); the correction
// x^ + d is written to the E slots and accumulated into dx / du.
__device__ __forceinline__ void lk_forward(const DevConst *dcp, double *wsb, int refine)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    const int odx = refine ? O_EDX : O_DX, odu = refine ? O_EDU : O_DU;
    double dxa[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) dxa[i] = 0.0;
#pragma unroll
    for (int i = 0; i < NX; ++i) W[odx + i * SXL] = 0.0;
    for (int k = 0; k < N; ++k) {
        const int kb = O_K + k * NU * NA;
        double kr[NU][NA], kk[NU], xk[NX], uk[NU], c[NX];
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            kk[a] = W[O_KK + k * NU + a];
#pragma unroll
            for (int j = 0; j < NA; ++j) kr[a][j] = W[kb + a * NA + j];
        }
        ldv(W, O_X, k, NX, xk);
        ldv(W, O_U, k, NU, uk);
        if (refine) ldv(W, O_DD, k + 1, NX, c);     // d_{k+1}
        else ldv(W, O_CC, k, NX, c);
        double du[NU];
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            double acc = kk[a];
#pragma unroll
            for (int j = 0; j < NA; ++j) acc += kr[a][j] * dxa[j];
            du[a] = acc;
        }
        double nx[NX], bd[NX];
        A_times(M, xk, uk, dxa, nx);
        B_times(M, xk, du, bd);
        double outx[NX];
        if (refine) {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                dxa[i] = nx[i] + bd[i];
                outx[i] = dxa[i] + c[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                dxa[i] = nx[i] + bd[i] + c[i];
                outx[i] = dxa[i];
            }
        }
#pragma unroll
        for (int a = 0; a < NU; ++a) dxa[NX + a] = du[a];
        stv(W, odx, k + 1, NX, outx);
        stv(W, odu, k, NU, du);
        if (refine) {
#pragma unroll
            for (int i = 0; i < NX; ++i) W[O_DX + i * SXL + k + 1] = W[O_DX + i * SXL + k + 1] + outx[i];
#pragma unroll
            for (int a = 0; a < NU; ++a) W[O_DU + a * SXL + k] = W[O_DU + a * SXL + k] + du[a];
        }
    }
}

// ---- costate recursion: lam+_{k-1} = (H_xx + Sigma + dw) dx_k + H_xu du_k + h_x + A^T lam+_k
__device__ __forceinline__ void lk_adjoint(const DevConst *dcp, double *wsb, double s, double mu, double dw, int refine,
                                        int lsq)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    Inst I;
    load_inst(W, I);
    const int odx = refine ? O_EDX : O_DX, odu = refine ? O_EDU : O_DU, olp = refine ? O_ELP : O_LP;
    double lp[NX];
    {
        // terminal: lam+_{N-1} = P_N dx_N + p_N  (P_N diagonal, closed form)
        double dxN[NX], pd[NX];
        ldv(W, odx, N, NX, dxN);
        pn_diag(D, M, W, N, s, mu, dw, lsq, pd);
#pragma unroll
        for (int i = 0; i < NX; ++i)
            lp[i] = (refine ? (double)W[O_RQ + i * SXL + N] : (double)W[O_PN + i]) + pd[i] * dxN[i];
        stv(W, olp, N - 1, NX, lp);
    }
    Attitude at;
    if (!lsq) load_att(W, M, at);
    for (int k = N - 1; k >= 1; --k) {
        double xk[NX], uk[NU], dx[NX], du[NU], h[NX], o[NX];
        ldv(W, O_X, k, NX, xk);
        ldv(W, O_U, k, NU, uk);
        ldv(W, odx, k, NX, dx);
        ldv(W, odu, k, NU, du);
        double sgw[3] = {0, 0, 0}, gbw[3] = {0, 0, 0};
        if (!lsq)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                bar(xk[10 + c], D.wlo, D.whi, W[O_ZLW + c * SXL + k], W[O_ZUW + c * SXL + k], mu, gbw[c], sgw[c]);
        if (refine) {
            ldv(W, O_RQ, k, NX, h);
        } else {
            grad_xs(M, at, I, W[O_WK + k], s, xk, h);
#pragma unroll
            for (int c = 0; c < 3; ++c)
                h[10 + c] += lsq ? (-(double)W[O_ZLW + c * SXL + k] + (double)W[O_ZUW + c * SXL + k]) : gbw[c];
        }
        if (lsq) {
#pragma unroll
            for (int i = 0; i < NX; ++i) o[i] = (1.0 + dw) * dx[i];
        } else {
            double lk[NX];
            ldv(W, O_LAM, k, NX, lk);
            StageHess H;
            stage_hessian(M, at, s, W[O_WK + k], xk, uk, lk, H);
            Hxx_times(H, dx, o);
            const double sdu = du[0] + du[1] + du[2] + du[3];
#pragma unroll
            for (int r = 0; r < 4; ++r) o[6 + r] += H.qu[r] * sdu;
#pragma unroll
            for (int i = 0; i < NX; ++i) o[i] += dw * dx[i];
#pragma unroll
            for (int c = 0; c < 3; ++c) o[10 + c] += sgw[c] * dx[10 + c];
        }
        double atl[NX];
        At_times(M, xk, uk, lp, atl);
#pragma unroll
        for (int i = 0; i < NX; ++i) lp[i] = h[i] + o[i] + atl[i];
        stv(W, olp, k - 1, NX, lp);
        if (refine) {
#pragma unroll
            for (int i = 0; i < NX; ++i) W[O_LP + i * SXL + k - 1] = W[O_LP + i * SXL + k - 1] + lp[i];
        }
    }
    if (refine) {
        // lam+_{N-1} correction accumulated last (it was needed unaccumulated above)
#pragma unroll
        for (int i = 0; i < NX; ++i) W[O_LP + i * SXL + N - 1] = W[O_LP + i * SXL + N - 1] + W[O_ELP + i * SXL + N - 1];
    }
}

// ---- refinement right-hand side: forward defect propagation d_{k+1} = A_k d_k + r_c,k (d_0 = 0).
// Substituting x = x^ + d removes the dynamics residual from the system, so the backward vector recursion
// needs only the gains K_k, chol(Q_uu,k) and closed-form stage Hessian products (no stored P):
//   h^_x = r_q + (H_xx + Sigma + dw) d,  h^_u = r_r + H_ux d,  p_N = r_q,N + P_N d_N.
__device__ __forceinline__ void lk_defect(const DevConst *dcp, double *wsb)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    double d[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) d[i] = 0.0;
    for (int k = 0; k < N; ++k) {
        double xk[NX], uk[NU], c[NX], ad[NX];
        ldv(W, O_X, k, NX, xk);
        ldv(W, O_U, k, NU, uk);
        ldv(W, O_RC, k, NX, c);
        A_times(M, xk, uk, d, ad);
#pragma unroll
        for (int i = 0; i < NX; ++i) d[i] = ad[i] + c[i];
        stv(W, O_DD, k + 1, NX, d);
    }
}

__device__ __forceinline__ void lk_backward_refine(const DevConst *dcp, double *wsb, double s, double mu, double dw)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    Attitude at;
    load_att(W, M, at);
    double p[NA];
    {
        double dN[NX], pd[NX];
        ldv(W, O_DD, N, NX, dN);
        pn_diag(D, M, W, N, s, mu, dw, 0, pd);
#pragma unroll
        for (int i = 0; i < NX; ++i) p[i] = W[O_RQ + i * SXL + N] + pd[i] * dN[i];
#pragma unroll
        for (int a = 0; a < NU; ++a) p[NX + a] = 0.0;
    }
    for (int k = N - 1; k >= 0; --k) {
        double xk[NX], uk[NU], hx[NX], hu[NU];
        ldv(W, O_X, k, NX, xk);
        ldv(W, O_U, k, NU, uk);
#pragma unroll
        for (int a = 0; a < NU; ++a) hu[a] = W[O_RR + a * SXL + k];
        if (k >= 1) {
            double d[NX], lk[NX], o[NX];
            ldv(W, O_DD, k, NX, d);
            ldv(W, O_LAM, k, NX, lk);
            ldv(W, O_RQ, k, NX, hx);
            StageHess H;
            stage_hessian(M, at, s, W[O_WK + k], xk, uk, lk, H);
            Hxx_times(H, d, o);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                double gb, sg;
                bar(xk[10 + c], D.wlo, D.whi, W[O_ZLW + c * SXL + k], W[O_ZUW + c * SXL + k], mu, gb, sg);
                o[10 + c] += sg * d[10 + c];
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) hx[i] += o[i] + dw * d[i];
            const double qd = H.qu[0] * d[6] + H.qu[1] * d[7] + H.qu[2] * d[8] + H.qu[3] * d[9];
#pragma unroll
            for (int a = 0; a < NU; ++a) hu[a] += qd;
        } else {
#pragma unroll
            for (int i = 0; i < NX; ++i) hx[i] = 0.0;
        }
        double gx[NX], gu[NU], bt[NU];
        At_times(M, xk, uk, p, gx);
        Bt_times(M, xk, p, bt);
#pragma unroll
        for (int i = 0; i < NX; ++i) gx[i] += hx[i];
#pragma unroll
        for (int a = 0; a < NU; ++a) gu[a] = bt[a] + p[NX + a] + hu[a];
        double L[10];
#pragma unroll
        for (int e = 0; e < 10; ++e) L[e] = W[O_L + k * 10 + e];
        double iL[4];
        chol_inv_diag(L, iL);
        double b0 = gu[0], b1 = gu[1], b2 = gu[2], b3 = gu[3];
        chol_fwd(L, iL, b0, b1, b2, b3);
        chol_bwd(L, iL, b0, b1, b2, b3);
        W[O_KK + k * NU + 0] = -b0; W[O_KK + k * NU + 1] = -b1;
        W[O_KK + k * NU + 2] = -b2; W[O_KK + k * NU + 3] = -b3;
        const int kb = O_K + k * NU * NA;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            double acc = (i < NX) ? gx[i] : 0.0;
#pragma unroll
            for (int a = 0; a < NU; ++a) acc += W[kb + a * NA + i] * gu[a];
            p[i] = acc;
        }
    }
}

// ---- KKT residual of the Newton system at (dx, du, lam+): writes r_q / r_r / r_c, returns IPOPT's ratio
__device__ __forceinline__ double lk_residual(const DevConst *dcp, double *wsb, double s, double mu, double dw)
{
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    Attitude at;
    load_att(W, M, at);
    Inst I;
    load_inst(W, I);
    double nres = 0, nsol = 0, nrhs = 0;
    for (int k = 0; k < N; ++k) {
        double xk[NX], uk[NU], up[NU], un[NU], dxk[NX], duk[NU], lpk[NX];
        ldv(W, O_X, k, NX, xk);
        ldv(W, O_U, k, NU, uk);
        ld_uprev(W, k, up);
        if (k + 1 < N) ldv(W, O_U, k + 1, NU, un);
        ldv(W, O_DX, k, NX, dxk);
        ldv(W, O_DU, k, NU, duk);
        ldv(W, O_LP, k, NX, lpk);
        StageHess H;
        double lk[NX];
        if (k >= 1) {
            ldv(W, O_LAM, k, NX, lk);
            stage_hessian(M, at, s, W[O_WK + k], xk, uk, lk, H);
        }
        // u rows
        double btl[NU], gu[NU];
        Bt_times(M, xk, lpk, btl);
        grad_us(M, s, k, N, uk, up, un, gu);
        double hux = 0.0;
        if (k >= 1) hux = H.qu[0] * dxk[6] + H.qu[1] * dxk[7] + H.qu[2] * dxk[8] + H.qu[3] * dxk[9];
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            double gb, sg;
            bar(uk[a], D.ulo, D.uhi, W[O_ZLU + a * SXL + k], W[O_ZUU + a * SXL + k], mu, gb, sg);
            const double R = s * (2 * M.wthrust + 2 * M.du_w) + sg + dw;
            double acc = R * duk[a];
            if (k + 1 < N) acc += 2 * M.du_w * s * (duk[a] - W[O_DU + a * SXL + k + 1]);
            if (k >= 1) acc += -2 * M.du_w * s * W[O_DU + a * SXL + k - 1];
            acc += hux;
            const double g = gu[a] + gb;
            acc += g + btl[a];
            W[O_RR + a * SXL + k] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(g));
            nsol = fmax(nsol, fabs(duk[a]));
        }
        // c rows
        double ax[NX], bd[NX], xn[NX], x1[NX];
        A_times(M, xk, uk, dxk, ax);
        B_times(M, xk, duk, bd);
        f_disc(M, xk, uk, xn);
        ldv(W, O_X, k + 1, NX, x1);
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const double c = xn[i] - x1[i];
            const double acc = c - W[O_DX + i * SXL + k + 1] + ax[i] + bd[i];
            W[O_RC + i * SXL + k] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(c));
            nsol = fmax(nsol, fabs(lpk[i]));
        }
        // x rows (k >= 1)
        if (k >= 1) {
            double o[NX], atl[NX], g[NX];
            Hxx_times(H, dxk, o);
            const double sdu = duk[0] + duk[1] + duk[2] + duk[3];
#pragma unroll
            for (int i = 0; i < 4; ++i) o[6 + i] += H.qu[i] * sdu;
            At_times(M, xk, uk, lpk, atl);
            grad_xs(M, at, I, W[O_WK + k], s, xk, g);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                double gb, sg;
                bar(xk[10 + c], D.wlo, D.whi, W[O_ZLW + c * SXL + k], W[O_ZUW + c * SXL + k], mu, gb, sg);
                g[10 + c] += gb;
                o[10 + c] += sg * dxk[10 + c];
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double acc = g[i] - W[O_LP + i * SXL + k - 1] + o[i] + dw * dxk[i] + atl[i];
                W[O_RQ + i * SXL + k] = acc;
                nres = fmax(nres, fabs(acc));
                nrhs = fmax(nrhs, fabs(g[i]));
                nsol = fmax(nsol, fabs(dxk[i]));
            }
        }
    }
    {
        // terminal x rows
        double xN[NX], dxN[NX], g[NX], o[NX];
        ldv(W, O_X, N, NX, xN);
        ldv(W, O_DX, N, NX, dxN);
        grad_xs(M, at, I, 0.0, s, xN, g);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            o[i] = (s * 2 * M.wrf + dw) * dxN[i];
            o[3 + i] = (s * 2 * M.wvf + dw) * dxN[3 + i];
        }
#pragma unroll
        for (int i = 6; i < 10; ++i) {
            double a = dw * dxN[i];
            if (M.wqf != 0.0)
#pragma unroll
                for (int j = 0; j < 4; ++j) a += s * M.wqf * (-2 * at.Sg[(i - 6) * 4 + j]) * dxN[6 + j];
            o[i] = a;
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double gb, sg;
            bar(xN[10 + c], D.wlo, D.whi, W[O_ZLW + c * SXL + N], W[O_ZUW + c * SXL + N], mu, gb, sg);
            g[10 + c] += gb;
            o[10 + c] = (s * 2 * M.wwf + sg + dw) * dxN[10 + c];
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const double acc = g[i] - W[O_LP + i * SXL + N - 1] + o[i];
            W[O_RQ + i * SXL + N] = acc;
            nres = fmax(nres, fabs(acc));
            nrhs = fmax(nrhs, fabs(g[i]));
            nsol = fmax(nsol, fabs(dxN[i]));
        }
    }
    if (nrhs + nres == 0.0) return nres;
    return nres / (fmin(nsol, 1e6 * nrhs) + nrhs);
}

// full Newton solve: factorisation + rollout + costates; 0 on inertia failure
__device__ __noinline__ int lk_newton_solve(const DevConst *dcp, double *wsb, double s, double mu, double dw, int lsq)
{
    LT_COUNT(12);
    LT_BEGIN;
    const int ok = lk_backward(dcp, wsb, s, mu, dw, lsq);
    LT_END(3);
    if (!ok) return 0;
    lk_forward(dcp, wsb, 0);
    LT_END(4);
    lk_adjoint(dcp, wsb, s, mu, dw, 0, lsq);
    LT_END(5);
    return 1;
}

__device__ void lk_dump(const DevConst *dcp, double *wsb, double *out)
{
    const int N = dconst(dcp).N;
    const LB W = make_lb(wsb);
    for (int e = 0; e < (N + 1) * NX; ++e) out[e] = W[O_DX + (e % NX) * SXL + e / NX];
    for (int e = 0; e < N * NU; ++e) out[(MAXN + 1) * NX + e] = W[O_DU + (e % NU) * SXL + e / NU];
    for (int e = 0; e < N * NX; ++e) out[(MAXN + 1) * NX + MAXN * NU + e] = W[O_LP + (e % NX) * SXL + e / NX];
}

// Newton step with iterative refinement (min 1, max 10 steps).  Returns 1 ok, 0 inertia failure.
__device__ __forceinline__ int lk_newton_step(const DevConst *dcp, double *wsb, double s, double mu, double dw, int &sweeps,
                                           double *ratios, double *dump_pre)
{
    const int N = dconst(dcp).N;
    const LB W = make_lb(wsb);
    LT_BEGIN;
    const int ok = lk_newton_solve(dcp, wsb, s, mu, dw, 0);
    LT_END(2);      // includes the solve's own phases 3-5: slot 2 - (3+4+5) = call overhead
    sweeps++;
    if (!ok) return 0;
    if (dump_pre) lk_dump(dcp, wsb, dump_pre);
    LT_END(11);
    double ratio = lk_residual(dcp, wsb, s, mu, dw);
    LT_END(6);
    ratios[0] = ratio; ratios[1] = -1; ratios[2] = -1; ratios[3] = 0;
    for (int step = 0; step < 10; ++step) {
        if (step >= 1 && ratio <= 1e-10) break;
        LT_COUNT(13);
        lk_defect(dcp, wsb);
        lk_backward_refine(dcp, wsb, s, mu, dw);
        LT_END(7);
        lk_forward(dcp, wsb, 1);
        LT_END(4);
        lk_adjoint(dcp, wsb, s, mu, dw, 1, 0);
        LT_END(5);
        sweeps++;
        const double nr = lk_residual(dcp, wsb, s, mu, dw);
        LT_END(6);
        if (step < 2) ratios[1 + step] = nr;
        ratios[3] += 1;
        if (!(nr < ratio)) {
            // revert the correction
            for (int k = 1; k <= N; ++k)
#pragma unroll
                for (int i = 0; i < NX; ++i) W[O_DX + i * SXL + k] = W[O_DX + i * SXL + k] - W[O_EDX + i * SXL + k];
            for (int k = 0; k < N; ++k) {
#pragma unroll
                for (int a = 0; a < NU; ++a) W[O_DU + a * SXL + k] = W[O_DU + a * SXL + k] - W[O_EDU + a * SXL + k];
#pragma unroll
                for (int i = 0; i < NX; ++i) W[O_LP + i * SXL + k] = W[O_LP + i * SXL + k] - W[O_ELP + i * SXL + k];
            }
            LT_END(0);
            break;
        }
        ratio = nr;
    }
    LT_END(11);
    return 1;
}

// ------------------------------------------------------------------------------------------------
// reward (rotor tips quad_model.py:239-276, collis_det solid_geometry.py:104-168, quad_policy.py:85-90)
__device__ inline void tip(const double *xt, const double *bx, const double *by, int r, double *out)
{
#pragma clang fp contract(off)
    double Cm[9];
    dcm(xt + 6, Cm);
#pragma unroll
    for (int i = 0; i < 3; ++i) out[i] = xt[i] + (Cm[0 * 3 + i] * bx[r] + Cm[1 * 3 + i] * by[r] + Cm[2 * 3 + i] * 0.0);
}

__device__ __forceinline__ double lk_reward(const DevConst *dcp, double *wsb, const double *g12)
{
#pragma clang fp contract(off)
    const cDevConst &D = dconst(dcp);
    const int N = D.N;
    const LB W = make_lb(wsb);
    double pt[4][3], cen[3];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) pt[i][j] = g12[i * 3 + j];
#pragma unroll
    for (int j = 0; j < 3; ++j) cen[j] = (pt[0][j] + pt[1][j] + pt[2][j] + pt[3][j]) / 4;
    Plane pl[4];
    Line ln[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double *b = pt[i], *c = pt[(i + 1) % 4];
        double v1[3], v2[3], cr[3], v3[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            pl[i].p1[j] = cen[j];
            v1[j] = b[j] - cen[j];
            v2[j] = c[j] - cen[j];
            v3[j] = c[j] - b[j];
        }
        cross3(v2, v1, cr);
        normv(cr, pl[i].normal);
        cross3(v1, pl[i].normal, cr);
        normv(cr, pl[i].n1);
        cross3(pl[i].normal, v2, cr);
        normv(cr, pl[i].n2);
        cross3(pl[i].normal, v3, cr);
        normv(cr, pl[i].n3);
        double d[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            ln[i].p1[j] = b[j];
            ln[i].p2[j] = c[j];
            d[j] = b[j] - c[j];
        }
        normv(d, ln[i].dir);
    }
    const double a = D.wing_len * 0.5 / sqrt(2.0);
    const double bx[4] = {a, -a, -a, a}, by[4] = {a, a, -a, -a};
    double col[4];
    for (int r = 0; r < 4; ++r) {
        double collision = 0.0;
        int first = -1;
        for (int t = 0; t < N; ++t) {
            double xt[NX], tp[3];
            ldv(W, O_X, t, NX, xt);
            tip(xt, bx, by, r, tp);
            const double d[3] = {tp[0] - cen[0], tp[1] - cen[1], tp[2] - cen[2]};
            if (dot3(pl[0].normal, d) < 0) { first = t; break; }
        }
        if (first > 0) {
            const int t = first;     // per lane
            double xt[NX], P1[3], P0[3];
#pragma unroll
            for (int i = 0; i < NX; ++i) xt[i] = W.ld_div(O_X + i * SXL + t);
            tip(xt, bx, by, r, P1);
#pragma unroll
            for (int i = 0; i < NX; ++i) xt[i] = W.ld_div(O_X + i * SXL + t - 1);
            tip(xt, bx, by, r, P0);
            double dir[3], dv[3] = {P1[0] - P0[0], P1[1] - P0[1], P1[2] - P0[2]};
            normv(dv, dir);
            double rel[3] = {P1[0] - pl[0].p1[0], P1[1] - pl[0].p1[1], P1[2] - pl[0].p1[2]};
            double tt = 1 / dot3(dir, pl[0].normal) * dot3(pl[0].normal, rel);
            double X[3] = {P1[0] - tt * dir[0], P1[1] - tt * dir[1], P1[2] - tt * dir[2]};
            double xc[3] = {X[0] - cen[0], X[1] - cen[1], X[2] - cen[2]};
            const double dmin = D.d_min;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                if (dot3(pl[p].n1, xc) > 0 && dot3(pl[p].n2, xc) > 0) {
                    double pv[3] = {pt[p][0] - X[0], pt[p][1] - X[1], pt[p][2] - X[2]};
                    if (dot3(pv, pl[p].n3) > 0) {
                        double mm = line_vertical(ln[0], X);
#pragma unroll
                        for (int l = 1; l < 4; ++l) mm = fmin(mm, line_vertical(ln[l], X));
                        double e = fmax(0.0, dmin - mm);
                        collision = -(e * e);
                    } else {
                        double mm = line_distance(ln[(p + 3) % 4], X);
                        mm = fmin(mm, line_distance(ln[p], X));
                        mm = fmin(mm, line_distance(ln[(p + 1) % 4], X));
                        collision = -2 * dmin * mm - dmin * dmin;
                    }
                }
            }
        }
        col[r] = collision;
    }
    double cs = 0.0;
    cs += col[0];
    cs += col[1];
    cs += col[2];
    cs += col[3];
    double path = 0.0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int t = N - 1 - p;
        double d[3] = {W[O_X + 0 * SXL + t] - cst(W, C_GOAL + 0), W[O_X + 1 * SXL + t] - cst(W, C_GOAL + 1),
                       W[O_X + 2 * SXL + t] - cst(W, C_GOAL + 2)};
        path += dot3(d, d);
    }
    return 1000 * cs - 0.5 * path + 100;
}

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void lane_kernel(KernelArgs A, const DevConst *dcp)
{
    const int lane = threadIdx.x;
    const int64_t inst = (int64_t)blockIdx.x * 64 + lane;
    const bool active = inst < A.n_inst;
    double *wsb = A.ws + (int64_t)blockIdx.x * BLOCK_DOUBLES;
    const cDevConst &D = dconst(dcp);
    const Model M = load_model(D);
    const int N = D.N;
    const LB W = make_lb(wsb);
    sPT = A.ptime ? A.ptime + (int64_t)blockIdx.x * 16 : nullptr;
    if (!active) return;
    LT_BEGIN;

    if (A.mode == MODE_REWARD) {
        for (int e = 0; e < (N + 1) * NX; ++e) W[O_X + (e % NX) * SXL + e / NX] = A.x_in[inst * (int64_t)(N + 1) * NX + e];
#pragma unroll
        for (int i = 0; i < 3; ++i) W[O_CST + C_GOAL + i] = A.goal[inst * 3 + i];
        A.reward_out[inst] = lk_reward(dcp, wsb, A.gate12 + inst * 12);
        return;
    }

    // ---- instance parameters (per mode), as ipm_kernel
    int64_t b = inst;
    int j = 0;
    if (A.mode == MODE_GRAD) {
        b = inst / 9;
        j = (int)(inst % 9);
    }
    double p3[3], a3[3], anorm, tt, q4[4];
    const double *ul = nullptr;
    if (A.mode == MODE_SOLVE || A.mode == MODE_OBJECTIVE) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            p3[i] = A.ptra[b * 3 + i];
            a3[i] = A.atra[b * 3 + i];
        }
        anorm = magni3(a3);
        tt = A.t[b];
        if (A.mode == MODE_OBJECTIVE) tt = round1_f64(tt);
        ul = A.ulast ? A.ulast + b * 4 : nullptr;
    } else {
        const float *o = A.dnn + b * 7;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            p3[i] = (double)o[i];
            a3[i] = (double)o[3 + i];
        }
        anorm = magni_f32(o + 3);
        if (A.mode == MODE_GETINPUT) {
            tt = (double)o[6];
            ul = A.ulast ? A.ulast + b * 4 : nullptr;
        } else {
            tt = round1_f32(o[6]);
            const double delta = 1e-3;
            if (j >= 1 && j <= 3) p3[j - 1] += delta;
            if (j >= 4 && j <= 6) {
                a3[j - 4] += delta;
                anorm = magni3(a3);
            }
            if (j >= 1 && j <= 6) ul = A.ulast ? A.ulast + b * 4 : nullptr;
            if (j == 7) tt = round1_f64((double)o[6] - 0.1);
            if (j == 8) tt = round1_f64((double)o[6] + 0.1);
        }
    }
    rd2quat(anorm, a3, q4);

    // ---- per-lane constants -> LDS
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        W[O_CST + C_GOAL + i] = A.goal[b * 3 + i];
        W[O_CST + C_PTRA + i] = p3[i];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) W[O_CST + C_UL + a] = ul ? ul[a] : 0.0;
    {
        double Rt[9], Rg[9], St[16], Sg[16];
        dcm(q4, Rt);
        attitude_form(Rt, St);
        const double qg[4] = {1, 0, 0, 0};
        dcm(qg, Rg);
        attitude_form(Rg, Sg);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            W[O_CST + C_ST + i] = St[i];
            W[O_CST + C_SG + i] = Sg[i];
        }
        W[O_CST + C_TRT] = Rt[0] + Rt[4] + Rt[8];
        W[O_CST + C_TRG] = Rg[0] + Rg[4] + Rg[8];
    }
    // ---- initial point (quad_OC.py:142,158: u = 1.22 projected into the relaxed box, x = 0)
    {
        const double umid = 0.5 * (D.u_lb + D.u_ub);
        const double wmid = 0.5 * (D.w_lb + D.w_ub);
        double pl = fmin(1e-2 * fmax(1.0, fabs(D.ulo)), 1e-2 * (D.uhi - D.ulo));
        double pu = fmin(1e-2 * fmax(1.0, fabs(D.uhi)), 1e-2 * (D.uhi - D.ulo));
        const double uinit = fmin(fmax(umid, D.ulo + pl), D.uhi - pu);
        pl = fmin(1e-2 * fmax(1.0, fabs(D.wlo)), 1e-2 * (D.whi - D.wlo));
        pu = fmin(1e-2 * fmax(1.0, fabs(D.whi)), 1e-2 * (D.whi - D.wlo));
        const double winit = fmin(fmax(wmid, D.wlo + pl), D.whi - pu);
        for (int k = 0; k <= N; ++k) {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                double v = 0.0;
                if (k == 0) v = A.ini[b * NX + i];
                else if (i >= 10) v = winit;
                W[O_X + i * SXL + k] = v;
                W[O_DX + i * SXL + k] = 0.0;
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                W[O_ZLW + c * SXL + k] = (k >= 1) ? 1.0 : 0.0;
                W[O_ZUW + c * SXL + k] = (k >= 1) ? 1.0 : 0.0;
            }
            const double dtk = M.dt * k - tt;
            W[O_WK + k] = D.tra_w_peak * exp(-D.tra_w_decay * dtk * dtk);
            if (k < N) {
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    W[O_U + a * SXL + k] = uinit;
                    W[O_ZLU + a * SXL + k] = 1.0;
                    W[O_ZUU + a * SXL + k] = 1.0;
                    W[O_DU + a * SXL + k] = 0.0;
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    W[O_LAM + i * SXL + k] = 0.0;
                    W[O_LP + i * SXL + k] = 0.0;
                }
            }
        }
    }
    // ---- gradient-based objective scaling
    double s = 1.0;
    {
        Attitude at;
        load_att(W, M, at);
        Inst I;
        load_inst(W, I);
        double gm = 0.0;
        for (int k = 0; k < N; ++k) {
            double x1[NX], g[NX], uk[NU], up[NU], un[NU], gu[NU];
            ldv(W, O_X, k + 1, NX, x1);
            grad_xs(M, at, I, (k + 1 < N) ? (double)W[O_WK + k + 1] : 0.0, 1.0, x1, g);
#pragma unroll
            for (int i = 0; i < NX; ++i) gm = fmax(gm, fabs(g[i]));
            ldv(W, O_U, k, NU, uk);
            ld_uprev(W, k, up);
            if (k + 1 < N) ldv(W, O_U, k + 1, NU, un);
            grad_us(M, 1.0, k, N, uk, up, un, gu);
#pragma unroll
            for (int a = 0; a < NU; ++a) gm = fmax(gm, fabs(gu[a]));
        }
        if (gm > 100.0) s = fmax(100.0 / gm, 1e-8);
    }
    int iters = 0, sweeps = 0, trials = 0;
    double mu = D.mu_init;
    // ---- least-squares constraint multipliers
    if (D.lsq_mult_init) {
        const int ok = lk_newton_solve(dcp, wsb, s, mu, 0.0, 1);
        sweeps++;
        if (ok) {
            double mx = 0.0;
            for (int k = 0; k < N; ++k)
#pragma unroll
                for (int i = 0; i < NX; ++i) mx = fmax(mx, fabs(W[O_LP + i * SXL + k]));
            if (mx <= 1e3)
                for (int k = 0; k < N; ++k)
#pragma unroll
                    for (int i = 0; i < NX; ++i) W[O_LAM + i * SXL + k] = W[O_LP + i * SXL + k];
        }
    }

    double tau = fmax(0.99, 1.0 - mu);
    int nfilt = 0;
    double theta_max = -1, theta_min = -1;
    double dw_last = 0.0;
    int acc_count = 0;
    int status = ST_MAXITER;
    int tiny_flag = 0;
    const double eps = 2.220446049250313e-16;

    LT_END(0);
    // Inertia-correction retries are folded into the main loop (a retrying lane re-enters the loop
    // without redoing the error / barrier update), so one lane's retry runs in the same Newton-solve
    // pass as the other lanes' next iteration instead of serialising the whole wave behind it.
    int retrying = 0;
    double dw_try = 0.0, e0 = 0.0;
    for (int it = 0; it <= D.max_iter; ++it) {
      if (!retrying) {
        LT_COUNT(15);
        Errs E = lk_errors(dcp, wsb, s, mu);
        LT_END(1);
        e0 = err_val(E, 0);
        if (!isfinite(e0)) { status = ST_NONFINITE; break; }
        if (e0 <= D.tol && E.dinf / s <= 1.0 && E.pinf <= 1e-4 && E.c0 / s <= 1e-4) {
            status = ST_SOLVED;
            break;
        }
        if (e0 <= D.acceptable_tol && E.dinf / s <= 1e10 && E.pinf <= 1e-2 && E.c0 / s <= 1e-2) {
            if (++acc_count >= D.acceptable_iter) { status = ST_ACCEPTABLE; break; }
        } else {
            acc_count = 0;
        }
        if (it == D.max_iter) { status = ST_MAXITER; break; }
        // monotone barrier update
        {
            const double mu_min = D.tol / 10.0;
            int done_tiny = 0;
            for (;;) {
                const double emu = err_val(E, 1);
                if (!(emu <= 10.0 * mu || tiny_flag)) break;
                const double nmu = fmax(mu_min, fmin(0.2 * mu, pow(mu, 1.5)));
                if (nmu == mu) {
                    if (tiny_flag) done_tiny = 1;
                    break;
                }
                mu = nmu;
                tau = fmax(0.99, 1.0 - mu);
                nfilt = 0;
                tiny_flag = 0;
                E = lk_errors(dcp, wsb, s, mu);
            }
            if (done_tiny) { status = ST_TINY; break; }
        }
        dw_try = 0.0;
      }
        // search direction with inertia correction (IPOPT: first trial dw = 0, then dw_last/3 or 1e-4,
        // growing by 8 (100 without history) until the factorisation has the right inertia)
        double ratios[4] = {0, 0, 0, 0};
        double *dpre = (A.dump && it == A.dump_it && !A.dump_refine) ? A.dump + inst * (int64_t)DUMP_W : nullptr;
        const int ok = lk_newton_step(dcp, wsb, s, mu, dw_try, sweeps, ratios, dpre);
        if (!ok) {
            if (dw_try == 0.0) dw_try = (dw_last == 0.0) ? 1e-4 : fmax(1e-20, dw_last / 3.0);
            else dw_try *= (dw_last == 0.0) ? 100.0 : 8.0;
            if (dw_try > 1e40) { status = ST_REG_FAIL; break; }
            retrying = 1;
            --it;
            continue;
        }
        retrying = 0;
        const double dw = dw_try;
        if (dw > 0.0) dw_last = dw;
        if (A.dump && it == A.dump_it && A.dump_refine) lk_dump(dcp, wsb, A.dump + inst * (int64_t)DUMP_W);
        _lt0 = sPT ? __builtin_amdgcn_s_memtime() : 0ull;
        // fraction to boundary, alpha_z, directional derivative, tiny-step measure
        double amax = 1.0, az = 1.0, gBD = 0.0, rel = 0.0;
        {
            Attitude at;
            load_att(W, M, at);
            Inst I;
            load_inst(W, I);
            double up[NU], uk[NU], un[NU];
            ld_uprev(W, 0, up);
            ldv(W, O_U, 0, NU, uk);
            for (int k = 0; k < N; ++k) {
                if (k + 1 < N) ldv(W, O_U, k + 1, NU, un);
                double gu[NU];
                grad_us(M, s, k, N, uk, up, un, gu);
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    const double v = uk[a], d = W[O_DU + a * SXL + k];
                    const double sl = v - D.ulo, su = D.uhi - v;
                    if (d < 0) amax = fmin(amax, -tau * sl / d);
                    if (d > 0) amax = fmin(amax, tau * su / d);
                    const double zl = W[O_ZLU + a * SXL + k], zu = W[O_ZUU + a * SXL + k];
                    const double dzl = mu / sl - zl - zl / sl * d;
                    const double dzu = mu / su - zu + zu / su * d;
                    if (dzl < 0) az = fmin(az, -tau * zl / dzl);
                    if (dzu < 0) az = fmin(az, -tau * zu / dzu);
                    double gb, sg;
                    bar(v, D.ulo, D.uhi, 0, 0, mu, gb, sg);
                    gBD += (gu[a] + gb) * d;
                    rel = fmax(rel, fabs(d) / (1.0 + fabs(v)));
                }
                const int k1 = k + 1;
                double x1[NX], g[NX];
                ldv(W, O_X, k1, NX, x1);
                grad_xs(M, at, I, (k1 < N) ? (double)W[O_WK + k1] : 0.0, s, x1, g);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const double v = x1[10 + c], d = W[O_DX + (10 + c) * SXL + k1];
                    const double sl = v - D.wlo, su = D.whi - v;
                    if (d < 0) amax = fmin(amax, -tau * sl / d);
                    if (d > 0) amax = fmin(amax, tau * su / d);
                    const double zl = W[O_ZLW + c * SXL + k1], zu = W[O_ZUW + c * SXL + k1];
                    const double dzl = mu / sl - zl - zl / sl * d;
                    const double dzu = mu / su - zu + zu / su * d;
                    if (dzl < 0) az = fmin(az, -tau * zl / dzl);
                    if (dzu < 0) az = fmin(az, -tau * zu / dzu);
                    double gb, sg;
                    bar(v, D.wlo, D.whi, 0, 0, mu, gb, sg);
                    g[10 + c] += gb;
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    const double d = W[O_DX + i * SXL + k1];
                    gBD += g[i] * d;
                    rel = fmax(rel, fabs(d) / (1.0 + fabs(x1[i])));
                }
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    up[a] = uk[a];
                    uk[a] = un[a];
                }
            }
        }
        const Merit m0 = lk_merit(dcp, wsb, s, mu, 0.0);
        const double th0 = m0.theta, ph0 = m0.phi;
        if (theta_max < 0) {
            theta_max = 1e4 * fmax(1.0, th0);
            theta_min = 1e-4 * fmax(1.0, th0);
        }
        double alpha = amax;
        int accepted = 0;
        const int is_tiny = (rel < 10.0 * eps) && (th0 <= 1e-4);
        double tht = 0, pht = 0;
        if (is_tiny) {
            accepted = 1;
            tiny_flag = 1;
        } else {
            double amin_base = 1e-5;
            if (gBD < 0) {
                amin_base = fmin(1e-5, 1e-8 * th0 / (-gBD));
                if (th0 <= theta_min) amin_base = fmin(amin_base, pow(th0, 1.1) / pow(-gBD, 2.3));
            }
            const double alpha_min = 0.05 * amin_base;
            for (;;) {
                LT_COUNT(14);
                const Merit mt = lk_merit(dcp, wsb, s, mu, alpha);
                tht = mt.theta;
                pht = mt.phi;
                trials++;
                int acc = mt.ok && !(tht > theta_max);
                if (acc) {
                    const int ftype = (gBD < 0) && (alpha * pow(-gBD, 2.3) > pow(th0, 1.1));
                    if (ftype && th0 <= theta_min) {
                        acc = (pht - ph0 - 1e-8 * alpha * gBD) <= 10.0 * eps * fabs(ph0);
                    } else {
                        int objinc_ok = 1;
                        if (pht > ph0) {
                            const double basval = (fabs(ph0) > 10.0) ? log10(fabs(ph0)) : 1.0;
                            if (log10(pht - ph0) > 5.0 + basval) objinc_ok = 0;
                        }
                        acc = objinc_ok && (((tht - (1.0 - 1e-5) * th0) <= 10.0 * eps * fabs(th0)) ||
                                            ((pht - ph0 + 1e-8 * th0) <= 10.0 * eps * fabs(ph0)));
                    }
                }
                if (acc) {
                    for (int f = 0; f < nfilt; ++f)
                        if (!(tht <= W[O_FT + f] || pht <= W[O_FP + f])) { acc = 0; break; }
                }
                if (acc) { accepted = 1; break; }
                alpha *= 0.5;
                if (alpha < alpha_min) break;
            }
            if (accepted) {
                const int ftype = (gBD < 0) && (alpha * pow(-gBD, 2.3) > pow(th0, 1.1));
                const int armijo = (pht - ph0 - 1e-8 * alpha * gBD) <= 10.0 * eps * fabs(ph0);
                if (!ftype || !armijo) {
                    const double nt = (1.0 - 1e-5) * th0, np = ph0 - 1e-8 * th0;
                    int wi = 0;
                    for (int f = 0; f < nfilt; ++f) {
                        const double ft = W[O_FT + f], fp = W[O_FP + f];
                        if (!(ft >= nt && fp >= np)) {
                            W.st_div(O_FT + wi, ft);
                            W.st_div(O_FP + wi, fp);
                            wi++;
                        }
                    }
                    if (wi < FMAX) {
                        W.st_div(O_FT + wi, nt);
                        W.st_div(O_FP + wi, np);
                        wi++;
                    }
                    nfilt = wi;
                }
            }
        }
        LT_END(8);
        if (A.trace && it < A.trace_iters) {
            double *tr = A.trace + (inst * (int64_t)A.trace_iters + it) * TRACE_W;
            tr[0] = mu; tr[1] = e0; tr[2] = th0; tr[3] = ph0; tr[4] = gBD; tr[5] = amax; tr[6] = az;
            tr[7] = alpha; tr[8] = dw; tr[9] = accepted; tr[10] = nfilt; tr[11] = sweeps;
            tr[12] = ratios[0]; tr[13] = ratios[1]; tr[14] = ratios[2]; tr[15] = ratios[3];
        }
        if (!accepted) {
            status = (e0 <= D.acceptable_tol) ? ST_ACCEPTABLE : ST_LS_FAIL;
            break;
        }
        if (is_tiny) alpha = amax;
        // accept: z with alpha_z (old slacks), lambda and primal with alpha, then kappa_sigma
        for (int k = 0; k < N; ++k) {
#pragma unroll
            for (int a = 0; a < NU; ++a) {
                const double v = W[O_U + a * SXL + k], d = W[O_DU + a * SXL + k];
                const double sl = v - D.ulo, su = D.uhi - v;
                const double zl = W[O_ZLU + a * SXL + k], zu = W[O_ZUU + a * SXL + k];
                const double nzl = zl + az * (mu / sl - zl - zl / sl * d);
                const double nzu = zu + az * (mu / su - zu + zu / su * d);
                const double nv = v + alpha * d;
                const double nsl = nv - D.ulo, nsu = D.uhi - nv;
                W[O_ZLU + a * SXL + k] = fmax(fmin(nzl, 1e10 * mu / nsl), mu / (1e10 * nsl));
                W[O_ZUU + a * SXL + k] = fmax(fmin(nzu, 1e10 * mu / nsu), mu / (1e10 * nsu));
                W[O_U + a * SXL + k] = nv;
            }
            const int k1 = k + 1;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double v = W[O_X + (10 + c) * SXL + k1], d = W[O_DX + (10 + c) * SXL + k1];
                const double sl = v - D.wlo, su = D.whi - v;
                const double zl = W[O_ZLW + c * SXL + k1], zu = W[O_ZUW + c * SXL + k1];
                const double nzl = zl + az * (mu / sl - zl - zl / sl * d);
                const double nzu = zu + az * (mu / su - zu + zu / su * d);
                const double nv = v + alpha * d;
                const double nsl = nv - D.wlo, nsu = D.whi - nv;
                W[O_ZLW + c * SXL + k1] = fmax(fmin(nzl, 1e10 * mu / nsl), mu / (1e10 * nsl));
                W[O_ZUW + c * SXL + k1] = fmax(fmin(nzu, 1e10 * mu / nsu), mu / (1e10 * nsu));
            }
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double l = W[O_LAM + i * SXL + k];
                W[O_LAM + i * SXL + k] = l + alpha * (W[O_LP + i * SXL + k] - l);
                W[O_X + i * SXL + k1] = W[O_X + i * SXL + k1] + alpha * W[O_DX + i * SXL + k1];
            }
        }
        iters++;
        LT_END(9);
    }
    // honor_original_bounds
    for (int k = 0; k < N; ++k) {
#pragma unroll
        for (int a = 0; a < NU; ++a) W[O_U + a * SXL + k] = fmin(fmax((double)W[O_U + a * SXL + k], D.u_lb), D.u_ub);
#pragma unroll
        for (int c = 0; c < 3; ++c)
            W[O_X + (10 + c) * SXL + k + 1] = fmin(fmax((double)W[O_X + (10 + c) * SXL + k + 1], D.w_lb), D.w_ub);
    }
    // ---- outputs
    if (A.x_out) {
        double *xo = A.x_out + inst * (int64_t)(N + 1) * NX;
        for (int k = 0; k <= N; ++k)
#pragma unroll
            for (int i = 0; i < NX; ++i) xo[k * NX + i] = W[O_X + i * SXL + k];
    }
    if (A.u_out) {
        double *uo = A.u_out + inst * (int64_t)N * NU;
        for (int k = 0; k < N; ++k)
#pragma unroll
            for (int a = 0; a < NU; ++a) uo[k * NU + a] = W[O_U + a * SXL + k];
    }
    if (A.lam_out) {
        double *lo = A.lam_out + inst * (int64_t)N * NX;
        for (int k = 0; k < N; ++k)
#pragma unroll
            for (int i = 0; i < NX; ++i) lo[k * NX + i] = W[O_LAM + i * SXL + k] / s;
    }
    if (A.cost_out) A.cost_out[inst] = lk_objective(dcp, wsb);
    LT_END(11);
    if (A.reward_out) A.reward_out[inst] = lk_reward(dcp, wsb, A.gate12 + b * 12);
    LT_END(10);
    if (A.status_out) A.status_out[inst] = status;
    if (A.iters_out) A.iters_out[inst] = iters;
    if (A.counters) {
        atomicAdd(&A.counters[0], (unsigned long long)iters);
        atomicAdd(&A.counters[1], (unsigned long long)sweeps);
        atomicAdd(&A.counters[2], (unsigned long long)trials);
    }
}

}  // namespace lane
}  // namespace lafse3
