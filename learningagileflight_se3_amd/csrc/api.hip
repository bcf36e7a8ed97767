// api.hip — extern "C" boundary of liblafse3.so (declared in include/lafse3.h).
//
// Host side only: argument checking, workspace management, kernel launches on the caller's stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "lafse3.h"

namespace lafse3 {
struct KernelArgs;
}

// kernels (#included so the whole library is one translation unit)
#include "ipm_kernel.hip"   // wave-per-instance solver (the only variant; params.variant must be WAVE)
#include "moving.hip"       // traversal-time fixed point of the moving-gate loop

namespace {

thread_local std::string g_err;

int fail(int code, const char *what, hipError_t e = hipSuccess)
{
    char buf[512];
    if (e != hipSuccess)
        snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    else
        snprintf(buf, sizeof(buf), "%s", what);
    g_err = buf;
    return code;
}

}  // namespace

struct lafse3_ctx {
    int device = 0;
    lafse3_params prm{};
    double *ws = nullptr;
    double *rws = nullptr;               // restoration-phase workspace (RWS_SIZE per slot)
    int64_t ws_inst = 0;
    double *tmp = nullptr;          // rewards9 scratch for sol_gradient
    int64_t tmp_n = 0;
    double *tmp32 = nullptr;        // fp64 staging of the fp32 twin (lafse3_ocp_solve_f32)
    int64_t tmp32_n = 0;
    unsigned long long *counters = nullptr;   // [0..2] iteration / sweep / trial totals, [3] work-queue head,
                                              // [4] device error word (ipm_kernel.hip ERR_*: kept until
                                              // lafse3_check_device reports it), [5..6] restoration counts;
                                              // words N_COUNTERS.. are trajectory scoring's (lafse3_reward)
    int64_t slots = 0;                         // resident solver waves: CUs x 4 SIMDs x waves per SIMD
    unsigned *sched = nullptr;                 // sol_gradient probe queue (ipm_kernel.hip sched_next)
    int64_t sched_n = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    double *trace = nullptr;   // debug trace target (device), see lafse3_debug_trace
    int trace_iters = 0;
    double *dump = nullptr;
    int dump_it = -1, dump_refine = 0;
    unsigned long long *ptime = nullptr;
    int32_t *iters_rec = nullptr;        // lafse3_record_iters target (device)
    int64_t iters_cap = 0;               // its capacity in entries
    int64_t drop_push = -1;              // debug: lafse3_debug_drop_push
    // private stream of the context: the counters of the last solver launch are read (and its error word cleared)
    // here after ev1 has completed, never on the caller's launch stream, which the caller may have destroyed since
    hipStream_t aux = nullptr;
};

static size_t ws_doubles(int64_t n) { return (size_t)n * (size_t)lafse3::WS_SIZE; }
constexpr int N_COUNTERS = 7;   // KernelArgs::counters words
static int ensure_sched(lafse3_ctx *c, int64_t B);

extern "C" {

int lafse3_default_params(lafse3_params *p)
{
    if (!p) return fail(LAFSE3_EINVAL, "null params");
    std::memset(p, 0, sizeof(*p));
    p->mass = 0.5; p->Jx = 0.0023; p->Jy = 0.0023; p->Jz = 0.004;          // quad_policy.py:37
    p->arm_l = 0.35; p->c_tau = 0.0245; p->grav = 9.78; p->dt = 0.1;        // quad_model.py:37, quad_policy.py:43
    p->wrt = 5; p->wqt = 80; p->wthrust = 0.1; p->wrf = 5; p->wvf = 5; p->wqf = 0; p->wwf = 3;  // quad_policy.py:38
    p->tra_w_peak = 60; p->tra_w_decay = 10; p->du_weight = 1;             // quad_OC.py:145,150
    p->u_lb = 0; p->u_ub = 2 * 1.22;                                        // quad_policy.py:48-51
    p->w_lb = -3.141592653589793 / 2; p->w_ub = 3.141592653589793 / 2;      // quad_policy.py:47,50
    p->wing_len = 1.5; p->d_min = 0.2;                                      // quad_policy.py:19, solid_geometry.py:115
    p->horizon = 50;                                                        // quad_policy.py:17
    p->max_iter = 3000; p->tol = 1e-8; p->acceptable_tol = 1e-6; p->acceptable_iter = 15;  // IPOPT defaults
    p->mu_init = 0.1; p->bound_relax = 1e-8; p->lsq_mult_init = 1;
    p->variant = LAFSE3_VARIANT_WAVE;
    p->max_soc = 4;
    p->costate_option = 0;
    p->grad_mode = 0;
    p->restoration = 1;
    p->watchdog = 10;
    return LAFSE3_OK;
}

int64_t lafse3_workspace_bytes_per_instance(void)
{
    return (int64_t)((ws_doubles(1) + (size_t)lafse3::RWS_SIZE) * sizeof(double));
}

int lafse3_stream_create(int device, void **stream)
{
    if (!stream) return fail(LAFSE3_EINVAL, "null stream");
    *stream = nullptr;
    if (device < 0) {
        const hipError_t e = hipGetDevice(&device);
        if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipGetDevice", e);
    }
    int cus = 0, prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess || cus <= 0) {
        if (prev >= 0) (void)hipSetDevice(prev);
        return fail(LAFSE3_EDEVICE, "CU count", e);
    }
    // a CU-masked stream gets a hardware queue of its own (the runtime does not share masked queues); the mask
    // enables every CU, so the stream runs exactly as an ordinary one otherwise
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xffffffffu);
    if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
    hipStream_t st = nullptr;
    e = hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data());
    if (prev >= 0) (void)hipSetDevice(prev);   // the caller's current device (torch's) stays as it was
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipExtStreamCreateWithCUMask", e);
    *stream = (void *)st;
    return LAFSE3_OK;
}

int lafse3_stream_destroy(void *stream)
{
    if (!stream) return fail(LAFSE3_EINVAL, "null stream");
    const hipError_t e = hipStreamDestroy((hipStream_t)stream);
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipStreamDestroy", e);
    return LAFSE3_OK;
}

int lafse3_create(lafse3_ctx **ctx, int device)
{
    if (!ctx) return fail(LAFSE3_EINVAL, "null ctx");
    lafse3_ctx *c = new lafse3_ctx();
    hipError_t e;
    if (device < 0) {
        e = hipGetDevice(&c->device);
        if (e != hipSuccess) { delete c; return fail(LAFSE3_EDEVICE, "hipGetDevice", e); }
    } else {
        c->device = device;
    }
    e = hipSetDevice(c->device);
    if (e != hipSuccess) { delete c; return fail(LAFSE3_EDEVICE, "hipSetDevice", e); }
    lafse3_default_params(&c->prm);
    e = hipMalloc(&c->counters, 2 * N_COUNTERS * sizeof(unsigned long long));
    if (e != hipSuccess) { delete c; return fail(LAFSE3_EDEVICE, "hipMalloc counters", e); }
    {
        // zeroed on a private stream and waited for there (a device-wide synchronize would also wait for other
        // contexts' solver launches in flight); complete before this call returns, so before any launch on it
        hipStream_t zs = nullptr;
        e = hipStreamCreateWithFlags(&zs, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMemsetAsync(c->counters, 0, 2 * N_COUNTERS * sizeof(unsigned long long), zs);
        if (e == hipSuccess) e = hipStreamSynchronize(zs);
        if (zs) (void)hipStreamDestroy(zs);
    }
    if (e != hipSuccess) {
        (void)hipFree(c->counters);
        delete c;
        return fail(LAFSE3_EDEVICE, "hipMemset counters", e);
    }
    int cus = 0;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    if (e != hipSuccess || cus <= 0) {
        (void)hipFree(c->counters);
        delete c;
        return fail(LAFSE3_EDEVICE, "hipDeviceGetAttribute(CU count)", e);
    }
    c->slots = (int64_t)cus * 4;   // one wave per SIMD (ipm_kernel __launch_bounds__(64, 1))
    if ((e = hipEventCreate(&c->ev0)) != hipSuccess || (e = hipEventCreate(&c->ev1)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking)) != hipSuccess) {
        if (c->ev0) (void)hipEventDestroy(c->ev0);
        if (c->ev1) (void)hipEventDestroy(c->ev1);
        (void)hipFree(c->counters);
        delete c;
        return fail(LAFSE3_EDEVICE, "hipEventCreate / hipStreamCreate", e);
    }
    *ctx = c;
    return LAFSE3_OK;
}

int lafse3_destroy(lafse3_ctx *c)
{
    if (!c) return LAFSE3_OK;
    (void)hipSetDevice(c->device);
    if (c->ws) (void)hipFree(c->ws);
    if (c->rws) (void)hipFree(c->rws);
    if (c->tmp) (void)hipFree(c->tmp);
    if (c->counters) (void)hipFree(c->counters);
    if (c->tmp32) (void)hipFree(c->tmp32);
    if (c->sched) (void)hipFree(c->sched);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    delete c;
    return LAFSE3_OK;
}

static int check_params(const lafse3_params *p)
{
    if (p->horizon < 1 || p->horizon > LAFSE3_MAX_N) return fail(LAFSE3_EINVAL, "horizon must be in [1, 50]");
    if (!(p->u_ub > p->u_lb) || !(p->w_ub > p->w_lb)) return fail(LAFSE3_EINVAL, "empty bound box");
    if (p->variant != LAFSE3_VARIANT_WAVE)
        return fail(LAFSE3_EINVAL, "unknown kernel variant (the lane-per-instance variant was removed in 0.3)");
    if (!(p->dt > 0) || !(p->mass > 0) || !(p->Jx > 0) || !(p->Jy > 0) || !(p->Jz > 0))
        return fail(LAFSE3_EINVAL, "non-positive model constant");
    if (p->max_iter < 0 || !(p->tol > 0) || p->max_soc < 0) return fail(LAFSE3_EINVAL, "bad solver option");
    if (p->costate_option != 0 && p->costate_option != 1) return fail(LAFSE3_EINVAL, "costate_option must be 0 or 1");
    if (p->grad_mode != 0 && p->grad_mode != 1) return fail(LAFSE3_EINVAL, "grad_mode must be 0 (FD) or 1 (IFT)");
    if (p->restoration != 0 && p->restoration != 1) return fail(LAFSE3_EINVAL, "restoration must be 0 or 1");
    if (p->watchdog < 0) return fail(LAFSE3_EINVAL, "watchdog must be >= 0");
    return LAFSE3_OK;
}

int lafse3_set_params(lafse3_ctx *c, const lafse3_params *p)
{
    if (!c || !p) return fail(LAFSE3_EINVAL, "null argument");
    int rc = check_params(p);
    if (rc) return rc;
    c->prm = *p;
    return LAFSE3_OK;
}

int lafse3_get_params(const lafse3_ctx *c, lafse3_params *p)
{
    if (!c || !p) return fail(LAFSE3_EINVAL, "null argument");
    *p = c->prm;
    return LAFSE3_OK;
}

int lafse3_reserve(lafse3_ctx *c, int64_t n)
{
    if (!c || n < 0) return fail(LAFSE3_EINVAL, "bad reserve");
    if (n > 0) {   // the probe queue of a sol_gradient launch of up to n samples (n instances cover n / 9)
        const int rq = ensure_sched(c, n);
        if (rq) return rq;
    }
    if (n > c->slots) n = c->slots;   // persistent solver: one workspace slot per resident wave
    if (n <= c->ws_inst) return LAFSE3_OK;
    (void)hipSetDevice(c->device);
    if (c->ws) { (void)hipFree(c->ws); c->ws = nullptr; c->ws_inst = 0; }
    if (c->rws) { (void)hipFree(c->rws); c->rws = nullptr; }
    hipError_t e = hipMalloc(&c->ws, ws_doubles(n) * sizeof(double));
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMalloc workspace", e);
    e = hipMalloc(&c->rws, (size_t)n * lafse3::RWS_SIZE * sizeof(double));
    if (e != hipSuccess) {
        (void)hipFree(c->ws);
        c->ws = nullptr;
        return fail(LAFSE3_EDEVICE, "hipMalloc restoration workspace", e);
    }
    c->ws_inst = n;
    return LAFSE3_OK;
}

static int ensure_tmp(lafse3_ctx *c, int64_t n)
{
    if (n <= c->tmp_n) return LAFSE3_OK;
    if (c->tmp) (void)hipFree(c->tmp);
    c->tmp = nullptr;
    c->tmp_n = 0;
    hipError_t e = hipMalloc(&c->tmp, (size_t)n * sizeof(double));
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMalloc scratch", e);
    c->tmp_n = n;
    return LAFSE3_OK;
}

// probe queue of a sol_gradient launch of B samples: 2 NB + 1 counters + NB x B bucket slots
static int64_t sched_words(int64_t B) { return 2 * lafse3::SCHED_NB + 1 + lafse3::SCHED_NB * B; }

static int ensure_sched(lafse3_ctx *c, int64_t B)
{
    const int64_t n = sched_words(B);
    if (n <= c->sched_n) return LAFSE3_OK;
    if (c->sched) (void)hipFree(c->sched);
    c->sched = nullptr;
    c->sched_n = 0;
    hipError_t e = hipMalloc(&c->sched, (size_t)n * sizeof(unsigned));
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMalloc probe queue", e);
    c->sched_n = n;
    return LAFSE3_OK;
}

// rewards9 / status9 slots before a sol_gradient launch: NaN / ST_DEVICE_ERR, overwritten by every solve that
// runs, so a slot whose probe task was lost (ipm_kernel.hip sched_next) cannot pass for a result
__global__ void slots_init_kernel(double *R, int32_t *S, int64_t n)
{
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= n) return;
    R[e] = __builtin_nan("");
    if (S) S[e] = lafse3::ST_DEVICE_ERR;
}

static int launch(lafse3_ctx *c, lafse3::KernelArgs &A, hipStream_t st, int64_t sched_samples = 0)
{
    if (A.n_inst == 0) return LAFSE3_OK;
    if (!A.iters_out && c->iters_rec) {
        // slots the kernel writes: b * 9 + j for sol_gradient (both gradient modes), the instance index otherwise
        const int64_t need = (A.mode == lafse3::MODE_GRAD) ? sched_samples * 9 : A.n_inst;
        if (need > c->iters_cap) {
            char buf[160];
            snprintf(buf, sizeof(buf), "lafse3_record_iters buffer holds %lld entries, this launch writes %lld",
                     (long long)c->iters_cap, (long long)need);
            return fail(LAFSE3_EINVAL, buf);
        }
        A.iters_out = c->iters_rec;
    }
    // persistent grid: one workgroup per SIMD slot (fewer when the batch is smaller), workspace per workgroup
    const int64_t grid = A.n_inst < c->slots ? A.n_inst : c->slots;
    int rc = lafse3_reserve(c, grid);
    if (rc) return rc;
    A.persistent = 1;
    A.prm = c->prm;
    A.ws = c->ws;
    A.rws = c->rws;
    // trajectory scoring (MODE_REWARD) counts nothing and has its own queue head: it leaves the last solver
    // launch's counters, error word, timing events and stream alone
    const bool scoring = A.mode == lafse3::MODE_REWARD;
    A.counters = scoring ? c->counters + N_COUNTERS : c->counters;
    A.trace = c->trace;
    A.trace_iters = c->trace_iters;
    A.ptime = c->ptime;
    A.dump = c->dump;
    A.dump_it = c->dump_it;
    A.dump_refine = c->dump_refine;
    A.drop_push = c->drop_push;
    // every word but the device error word, which stays set until lafse3_check_device has reported it
    hipError_t e = hipMemsetAsync(A.counters, 0, lafse3::CNT_ERR * sizeof(unsigned long long), st);
    if (e == hipSuccess)
        e = hipMemsetAsync(A.counters + lafse3::CNT_ERR + 1, 0,
                           (N_COUNTERS - lafse3::CNT_ERR - 1) * sizeof(unsigned long long), st);
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMemsetAsync", e);
    A.sched = nullptr;
    if (sched_samples > 0) {
        rc = ensure_sched(c, sched_samples);
        if (rc) return rc;
        e = hipMemsetAsync(c->sched, 0, (size_t)sched_words(sched_samples) * sizeof(unsigned), st);
        if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMemsetAsync probe queue", e);
        A.sched = c->sched;
    }
    if (scoring) {
        hipLaunchKernelGGL(lafse3::ipm_kernel, dim3((unsigned)grid), dim3(64), 0, st, A);
        e = hipGetLastError();
        if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "scoring kernel launch", e);
        return LAFSE3_OK;
    }
    (void)hipEventRecord(c->ev0, st);
    hipLaunchKernelGGL(lafse3::ipm_kernel, dim3((unsigned)grid), dim3(64), 0, st, A);
    e = hipGetLastError();
    (void)hipEventRecord(c->ev1, st);
    c->timed = true;
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "solver kernel launch", e);
    return LAFSE3_OK;
}

static lafse3::KernelArgs blank_args()
{
    lafse3::KernelArgs A;
    std::memset(&A, 0, sizeof(A));
    return A;
}

int lafse3_ocp_solve(lafse3_ctx *c, int64_t B, const double *ini, const double *goal, const double *p_tra,
                     const double *a_tra, const double *t, const double *u_last, double *x, double *u, double *lam,
                     double *cost, int32_t *status, int32_t *iters, void *stream)
{
    if (!c || B < 0) return fail(LAFSE3_EINVAL, "bad ctx / batch");
    if (B > 0 && (!ini || !goal || !p_tra || !a_tra || !t)) return fail(LAFSE3_EINVAL, "null input");
    if (B > 0x7fffffffLL) return fail(LAFSE3_EINVAL, "batch too large for one launch");
    (void)hipSetDevice(c->device);
    lafse3::KernelArgs A = blank_args();
    A.mode = lafse3::MODE_SOLVE;
    A.n_inst = B;
    A.ini = ini; A.goal = goal; A.ptra = p_tra; A.atra = a_tra; A.t = t; A.ulast = u_last;
    A.x_out = x; A.u_out = u; A.lam_out = lam; A.cost_out = cost; A.status_out = status; A.iters_out = iters;
    return launch(c, A, (hipStream_t)stream);
}

// ---- fp32 twin of lafse3_ocp_solve: float inputs/outputs at the boundary, fp64 arithmetic inside (IPOPT's
// 1e-8 tolerance is below float32 resolution, so the solve itself cannot run in fp32)
__global__ void f32_to_f64_kernel(const float *in, double *out, int64_t n)
{
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e < n) out[e] = (double)in[e];
}

__global__ void f64_to_f32_kernel(const double *in, float *out, int64_t n)
{
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e < n) out[e] = (float)in[e];
}

static int convert(const void *in, void *out, int64_t n, bool to64, hipStream_t st)
{
    if (n == 0 || !in || !out) return LAFSE3_OK;
    const int tpb = 256;
    const unsigned g = (unsigned)((n + tpb - 1) / tpb);
    if (to64) hipLaunchKernelGGL(f32_to_f64_kernel, dim3(g), dim3(tpb), 0, st, (const float *)in, (double *)out, n);
    else hipLaunchKernelGGL(f64_to_f32_kernel, dim3(g), dim3(tpb), 0, st, (const double *)in, (float *)out, n);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? LAFSE3_OK : fail(LAFSE3_EDEVICE, "fp32/fp64 conversion launch", e);
}

int lafse3_ocp_solve_f32(lafse3_ctx *c, int64_t B, const float *ini, const float *goal, const float *p_tra,
                         const float *a_tra, const float *t, const float *u_last, float *x, float *u, float *lam,
                         float *cost, int32_t *status, int32_t *iters, void *stream)
{
    if (!c || B < 0) return fail(LAFSE3_EINVAL, "bad ctx / batch");
    if (B > 0 && (!ini || !goal || !p_tra || !a_tra || !t)) return fail(LAFSE3_EINVAL, "null input");
    if (B > 0x7fffffffLL) return fail(LAFSE3_EINVAL, "batch too large for one launch");
    if (B == 0) return LAFSE3_OK;
    (void)hipSetDevice(c->device);
    const int64_t N = c->prm.horizon;
    const int64_t nin = B * (13 + 3 + 3 + 3 + 1 + 4);
    const int64_t nx = x ? B * (N + 1) * 13 : 0, nu = u ? B * N * 4 : 0, nl = lam ? B * N * 13 : 0, nc = cost ? B : 0;
    const int64_t need = nin + nx + nu + nl + nc;
    if (need > c->tmp32_n) {
        if (c->tmp32) (void)hipFree(c->tmp32);
        c->tmp32 = nullptr;
        c->tmp32_n = 0;
        hipError_t e = hipMalloc(&c->tmp32, (size_t)need * sizeof(double));
        if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMalloc fp32 staging", e);
        c->tmp32_n = need;
    }
    double *d = c->tmp32;
    double *dini = d, *dgoal = dini + 13 * B, *dp = dgoal + 3 * B, *da = dp + 3 * B, *dt = da + 3 * B, *dul = dt + B;
    double *dx = dul + 4 * B, *du = dx + nx, *dl = du + nu, *dc = dl + nl;
    hipStream_t st = (hipStream_t)stream;
    int rc = 0;
    if ((rc = convert(ini, dini, 13 * B, true, st)) || (rc = convert(goal, dgoal, 3 * B, true, st)) ||
        (rc = convert(p_tra, dp, 3 * B, true, st)) || (rc = convert(a_tra, da, 3 * B, true, st)) ||
        (rc = convert(t, dt, B, true, st)) || (rc = convert(u_last, dul, u_last ? 4 * B : 0, true, st)))
        return rc;
    rc = lafse3_ocp_solve(c, B, dini, dgoal, dp, da, dt, u_last ? dul : nullptr, x ? dx : nullptr, u ? du : nullptr,
                          lam ? dl : nullptr, cost ? dc : nullptr, status, iters, stream);
    if (rc) return rc;
    if ((rc = convert(dx, x, nx, false, st)) || (rc = convert(du, u, nu, false, st)) ||
        (rc = convert(dl, lam, nl, false, st)) || (rc = convert(dc, cost, nc, false, st)))
        return rc;
    return LAFSE3_OK;
}

int lafse3_objective(lafse3_ctx *c, int64_t B, const double *ini, const double *goal, const double *gate12,
                     const double *p_tra, const double *a_tra, const double *t, const double *u_last, double *reward,
                     int32_t *status, void *stream)
{
    if (!c || B < 0) return fail(LAFSE3_EINVAL, "bad ctx / batch");
    if (B > 0 && (!ini || !goal || !gate12 || !p_tra || !a_tra || !t || !reward))
        return fail(LAFSE3_EINVAL, "null argument");
    (void)hipSetDevice(c->device);
    lafse3::KernelArgs A = blank_args();
    A.mode = lafse3::MODE_OBJECTIVE;
    A.n_inst = B;
    A.ini = ini; A.goal = goal; A.gate12 = gate12; A.ptra = p_tra; A.atra = a_tra; A.t = t; A.ulast = u_last;
    A.reward_out = reward; A.status_out = status;
    return launch(c, A, (hipStream_t)stream);
}

int lafse3_sol_gradient(lafse3_ctx *c, int64_t B, const double *ini, const double *goal, const double *gate12,
                        const float *dnn_out, const double *u_last, double *out8, double *rewards9, int32_t *status9,
                        void *stream)
{
    if (!c || B < 0) return fail(LAFSE3_EINVAL, "bad ctx / batch");
    if (B > 0 && (!ini || !goal || !gate12 || !dnn_out || !out8)) return fail(LAFSE3_EINVAL, "null argument");
    if (B * 9 > 0x7fffffffLL) return fail(LAFSE3_EINVAL, "batch too large for one launch");
    const bool ift = c && c->prm.grad_mode == 1;
    if (ift && u_last) return fail(LAFSE3_EINVAL, "grad_mode 1 (IFT) linearises the nominal solve: u_last must be NULL");
    if (B == 0) return LAFSE3_OK;
    (void)hipSetDevice(c->device);
    double *R = rewards9;
    if (!R) {
        int rc = ensure_tmp(c, B * 9);
        if (rc) return rc;
        R = c->tmp;
    }
    lafse3::KernelArgs A = blank_args();
    A.mode = lafse3::MODE_GRAD;
    A.n_inst = ift ? B * 3 : B * 9;   // IFT: nominal + the two t probes; slots of rewards9 / status9 unchanged
    A.ini = ini; A.goal = goal; A.gate12 = gate12; A.dnn = dnn_out; A.ulast = u_last;
    A.reward_out = R; A.status_out = status9;
    hipStream_t st = (hipStream_t)stream;
    {
        const int tpb = 256;
        hipLaunchKernelGGL(slots_init_kernel, dim3((unsigned)((9 * B + tpb - 1) / tpb)), dim3(tpb), 0, st, R, status9,
                           9 * B);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "slots_init_kernel launch", e);
    }
    int rc = launch(c, A, st, B);   // nominal solves first, then the probes longest-first (sched_next)
    if (rc) return rc;
    const int tpb = 256;
    hipLaunchKernelGGL(lafse3::assemble_kernel, dim3((unsigned)((B + tpb - 1) / tpb)), dim3(tpb), 0, st, B, R,
                       dnn_out, out8);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "assemble_kernel launch", e);
    return LAFSE3_OK;
}

int lafse3_get_input(lafse3_ctx *c, int64_t B, const double *ini, const double *goal, const double *u_last,
                     const float *dnn_out, double *u0, double *x, int32_t *status, void *stream)
{
    if (!c || B < 0) return fail(LAFSE3_EINVAL, "bad ctx / batch");
    if (B > 0 && (!ini || !goal || !dnn_out || !u0)) return fail(LAFSE3_EINVAL, "null argument");
    if (B == 0) return LAFSE3_OK;
    (void)hipSetDevice(c->device);
    const int N = c->prm.horizon;
    // full control trajectory goes to scratch; u0 is its first row (copied with a 2-D memcpy)
    int rc = ensure_tmp(c, B * (int64_t)N * 4);
    if (rc) return rc;
    lafse3::KernelArgs A = blank_args();
    A.mode = lafse3::MODE_GETINPUT;
    A.n_inst = B;
    A.ini = ini; A.goal = goal; A.dnn = dnn_out; A.ulast = u_last;
    A.u_out = c->tmp; A.x_out = x; A.status_out = status;
    hipStream_t st = (hipStream_t)stream;
    rc = launch(c, A, st);
    if (rc) return rc;
    hipError_t e = hipMemcpy2DAsync(u0, 4 * sizeof(double), c->tmp, (size_t)N * 4 * sizeof(double),
                                    4 * sizeof(double), (size_t)B, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMemcpy2DAsync", e);
    return LAFSE3_OK;
}

int lafse3_reward(lafse3_ctx *c, int64_t B, const double *x, const double *goal, const double *gate12, double *reward,
                  void *stream)
{
    if (!c || B < 0) return fail(LAFSE3_EINVAL, "bad ctx / batch");
    if (B > 0 && (!x || !goal || !gate12 || !reward)) return fail(LAFSE3_EINVAL, "null argument");
    if (B > 0x7fffffffLL) return fail(LAFSE3_EINVAL, "batch too large for one launch");
    if (B == 0) return LAFSE3_OK;
    (void)hipSetDevice(c->device);
    lafse3::KernelArgs A = blank_args();
    A.mode = lafse3::MODE_REWARD;
    A.n_inst = B;
    A.x_in = x; A.goal = goal; A.gate12 = gate12; A.reward_out = reward;
    // the same persistent launch as the solves: min(B, slots) workgroups, each with its own workspace slot
    const int32_t *keep = c->iters_rec;   // trajectory scoring records no iteration counts
    c->iters_rec = nullptr;
    const int rc = launch(c, A, (hipStream_t)stream);
    c->iters_rec = const_cast<int32_t *>(keep);
    return rc;
}

int lafse3_traversal_time(lafse3_ctx *c, int64_t B, const double *state, const double *final_point,
                          const double *gate12, const double *velo, double w, const float *dnn2_weights,
                          double *t_out, int32_t *iters, void *stream)
{
    if (!c || B < 0) return fail(LAFSE3_EINVAL, "bad ctx / batch");
    if (B > 0 && (!state || !final_point || !gate12 || !velo || !dnn2_weights || !t_out))
        return fail(LAFSE3_EINVAL, "null argument");
    if (B == 0) return LAFSE3_OK;
    (void)hipSetDevice(c->device);
    lafse3::TTArgs A;
    A.B = B;
    A.state = state; A.final_point = final_point; A.gate = gate12; A.velo = velo;
    A.w = w;
    A.weights = dnn2_weights;
    A.t_out = t_out;
    A.iters = iters;
    if (((uintptr_t)dnn2_weights & 15) != 0) return fail(LAFSE3_EINVAL, "dnn2_weights not 16-byte aligned");
    // one wave per episode, grid-stride: two rounds of resident waves (1 per SIMD at its register count)
    const int64_t grid = B < 2 * c->slots ? B : 2 * c->slots;
    hipLaunchKernelGGL(lafse3::traversal_time_kernel, dim3((unsigned)grid), dim3(64), 0, (hipStream_t)stream, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "traversal_time launch", e);
    return LAFSE3_OK;
}

int lafse3_dnn2_weight_count(void) { return lafse3::TT_NW; }

float lafse3_last_kernel_ms(const lafse3_ctx *c)
{
    if (!c || !c->timed) return -1.0f;
    float ms = -1.0f;
    if (hipEventSynchronize(c->ev1) != hipSuccess) return -1.0f;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.0f;
    return ms;
}

static int read_counters(lafse3_ctx *c, unsigned long long h[N_COUNTERS])
{
    // the counters are written by the last solver launch: wait for its end event (recorded on the launch stream,
    // which may be a non-blocking torch stream or one the caller has destroyed since), then copy on the context's
    // own stream -- not on the launch stream and not on the legacy default stream
    (void)hipSetDevice(c->device);
    hipError_t e = hipEventSynchronize(c->ev1);
    if (e == hipSuccess)
        e = hipMemcpyAsync(h, c->counters, N_COUNTERS * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->aux);
    if (e == hipSuccess) e = hipStreamSynchronize(c->aux);
    if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMemcpyAsync counters", e);
    if (h[lafse3::CNT_ERR]) {
        char buf[200];
        snprintf(buf, sizeof(buf), "device error word 0x%llx raised by a solver launch since the last lafse3_check_device%s",
                 h[lafse3::CNT_ERR],
                 (h[lafse3::CNT_ERR] & lafse3::ERR_PROBE_LOST)
                     ? ": a sol_gradient probe task was lost (its rewards9/status9 slot holds NaN / status 7)" : "");
        return fail(LAFSE3_EDEVICE, buf);
    }
    return LAFSE3_OK;
}

int lafse3_last_counters(lafse3_ctx *c, int64_t counters[3])
{
    if (!c || !counters) return fail(LAFSE3_EINVAL, "null argument");
    unsigned long long h[N_COUNTERS] = {};
    if (!c->timed) return fail(LAFSE3_EINVAL, "no solver launch on this context yet");
    const int rc = read_counters(c, h);
    for (int i = 0; i < 3; ++i) counters[i] = (int64_t)h[i];
    return rc;
}

int lafse3_last_resto_counters(lafse3_ctx *c, int64_t counters[2])
{
    if (!c || !counters) return fail(LAFSE3_EINVAL, "null argument");
    unsigned long long h[N_COUNTERS] = {};
    if (!c->timed) return fail(LAFSE3_EINVAL, "no solver launch on this context yet");
    const int rc = read_counters(c, h);
    counters[0] = (int64_t)h[lafse3::CNT_RESTO];
    counters[1] = (int64_t)h[lafse3::CNT_RESTO + 1];
    return rc;
}

int lafse3_check_device(lafse3_ctx *c)
{
    if (!c) return fail(LAFSE3_EINVAL, "null ctx");
    if (!c->timed) return LAFSE3_OK;
    unsigned long long h[N_COUNTERS] = {};
    const int rc = read_counters(c, h);
    if (rc != LAFSE3_OK && !h[lafse3::CNT_ERR]) return rc;   // the copy itself failed
    if (h[lafse3::CNT_ERR]) {   // reported: clear it for the launches that follow
        hipError_t e = hipMemsetAsync(c->counters + lafse3::CNT_ERR, 0, sizeof(unsigned long long), c->aux);
        if (e == hipSuccess) e = hipStreamSynchronize(c->aux);
        if (e != hipSuccess) return fail(LAFSE3_EDEVICE, "hipMemsetAsync error word", e);
    }
    return rc;
}

int lafse3_debug_drop_push(lafse3_ctx *c, int64_t sample)
{
    if (!c) return fail(LAFSE3_EINVAL, "null ctx");
    c->drop_push = sample;
    return LAFSE3_OK;
}

int lafse3_debug_trace(lafse3_ctx *c, double *buf, int iters)
{
    if (!c) return fail(LAFSE3_EINVAL, "null ctx");
    c->trace = buf;
    c->trace_iters = buf ? iters : 0;
    return LAFSE3_OK;
}

int lafse3_debug_timers(lafse3_ctx *c, uint64_t *buf)
{
    if (!c) return fail(LAFSE3_EINVAL, "null ctx");
    c->ptime = (unsigned long long *)buf;
    return LAFSE3_OK;
}

int lafse3_debug_dump(lafse3_ctx *c, double *buf, int it, int after_refine)
{
    if (!c) return fail(LAFSE3_EINVAL, "null ctx");
    c->dump = buf;
    c->dump_it = buf ? it : -1;
    c->dump_refine = after_refine;
    return LAFSE3_OK;
}

int lafse3_record_iters(lafse3_ctx *c, int32_t *buf, int64_t capacity)
{
    if (!c) return fail(LAFSE3_EINVAL, "null ctx");
    if (buf && capacity <= 0) return fail(LAFSE3_EINVAL, "record_iters: capacity must be > 0");
    c->iters_rec = buf;
    c->iters_cap = buf ? capacity : 0;
    return LAFSE3_OK;
}

const char *lafse3_last_error(void) { return g_err.c_str(); }

const char *lafse3_version(void) { return "lafse3 0.5.0 (gfx950)"; }

}  // extern "C"
