/*
 * lafse3.h — C ABI of the MI355X-native batched SE(3) MPC solve + gradient engine.
 *
 * Drop-in boundary for the optimal-control hot path of yanrui89/LearningAgileFlight_SE3:
 *
 *   lafse3_ocp_solve      replaces OCSys.ocSolver            quad_OC.py:104-212
 *                         (cost configured as run_quad does:  quad_policy.py:35-56, :74-77,
 *                          traversal cost quad_model.py:200-213, setTraCost quad_OC.py:98-101)
 *   lafse3_objective      replaces run_quad.objective         quad_policy.py:67-91
 *   lafse3_sol_gradient   replaces run_quad.sol_gradient      quad_policy.py:94-112
 *   lafse3_get_input      replaces run_quad.get_input         quad_policy.py:202-211
 *
 * Every array argument is a DEVICE pointer (HBM; e.g. a torch.cuda tensor's data_ptr()), owned by
 * the caller, row-major, contiguous.  B is the batch size.  N is params.horizon (<= LAFSE3_MAX_N).
 * The library keeps no global mutable state: all state is in the opaque context (device workspace,
 * parameters).  Calls on one context must not overlap, and a context must be used from ONE stream at a
 * time: the workspace, scratch and counters are shared by every call on it and each call runs on the
 * caller's stream (use one context per stream); distinct contexts are independent.
 *
 * Return codes: 0 ok; LAFSE3_EINVAL bad argument; LAFSE3_EDEVICE HIP error (message via
 * lafse3_last_error).  Per-instance solver outcome is reported in `status` (never aborts):
 *   0 solved (IPOPT tol), 1 solved to acceptable level, 2 max_iter, 3 line-search failure,
 *   4 non-finite, 5 tiny step, 6 inertia regularisation failed (in lafse3_sol_gradient's IFT mode also: the
 *   factorisation at the nominal optimum failed, so the p/a probe rewards fell back to the nominal reward),
 *   7 device error (a sol_gradient slot no solve wrote: reward NaN; lafse3_check_device reports it),
 *   8 restoration phase failed (its line search; IPOPT Restoration_Failed), 9 the restoration phase converged to
 *   a point that is not feasible for the original problem (IPOPT Infeasible_Problem_Detected).  After 8 and 9 the
 *   outputs hold the point where the restoration phase started.
 * Outputs are always written with the last iterate (the reference uses IPOPT's last iterate too).
 */
#ifndef LAFSE3_H
#define LAFSE3_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LAFSE3_NX 13
#define LAFSE3_NU 4
#define LAFSE3_MAX_N 50

#define LAFSE3_OK 0
#define LAFSE3_EINVAL (-1)
#define LAFSE3_EDEVICE (-2)

/* Problem + solver parameters.  Defaults (lafse3_default_params) equal the reference:
 * model quad_policy.py:37 + quad_model.py:37, weights quad_policy.py:38 + quad_OC.py:145,150,
 * bounds quad_policy.py:46-51, dt quad_policy.py:43, horizon quad_policy.py:17, winglen :19,
 * IPOPT 3.12 defaults for the solver options (quad_OC.py:170 sets only print options). */
typedef struct lafse3_params {
    double mass, Jx, Jy, Jz, arm_l, c_tau, grav, dt;
    double wrt, wqt, wthrust, wrf, wvf, wqf, wwf;
    double tra_w_peak, tra_w_decay, du_weight;
    double u_lb, u_ub, w_lb, w_ub;
    double wing_len, d_min;
    int32_t horizon;
    int32_t max_iter;
    double tol, acceptable_tol;
    int32_t acceptable_iter;
    double mu_init, bound_relax;
    int32_t lsq_mult_init;
    int32_t variant;          /* must be LAFSE3_VARIANT_WAVE (kept for ABI layout; LANE was removed in 0.3) */
    int32_t max_soc;          /* IPOPT max_soc (default 4): second-order corrections per line search */
    int32_t costate_option;   /* lam output of lafse3_ocp_solve: 0 = IPOPT lam_g (default, quad_OC.py:185-187),
                                 1 = PMP costates recomputed on the optimum (quad_OC.py:188-201) */
    int32_t grad_mode;        /* lafse3_sol_gradient: 0 = FD, the reference's 9 solves per sample (default,
                                 quad_policy.py:94-112); 1 = IFT: 3 solves (nominal, t -+ 0.1) and the six
                                 p/a probes R(p + 1e-3 e_i) replaced by R(xs + 1e-3 dxs_i), xs the nominal
                                 optimum and dxs_i its sensitivity to parameter i from the nominal solve's last
                                 KKT factorisation (implicit function theorem, one refinement sweep per
                                 parameter); requires u_last == NULL */
    int32_t restoration;      /* 1 (default): IPOPT's restoration phase after a failed line search (feasibility
                                 problem min rho ||p + n||_1 + eta/2 ||D_R (v - v_R)||^2, IpRestoPhase); 0: the solve
                                 ends there (status 3, or 1 at an acceptable point) as up to 0.4 */
    int32_t watchdog;         /* IPOPT watchdog_shortened_iter_trigger (default 10; 0 disables): after this many
                                 successive iterations whose line search rejected the first trial point, up to 3
                                 (watchdog_trial_iter_max) full steps are taken before the stored iterate resumes */
} lafse3_params;

/* Kernel variant: one NLP instance per 64-lane wavefront (the only one).  The value 0 (a lane-per-instance
 * variant up to 0.2) is rejected with LAFSE3_EINVAL. */
#define LAFSE3_VARIANT_WAVE 1

typedef struct lafse3_ctx lafse3_ctx;

/* Fill *p with the reference defaults.  Returns 0. */
int lafse3_default_params(lafse3_params *p);

/* Create a context bound to HIP device `device` (the caller's current device if < 0). */
int lafse3_create(lafse3_ctx **ctx, int device);
int lafse3_destroy(lafse3_ctx *ctx);
int lafse3_set_params(lafse3_ctx *ctx, const lafse3_params *p);
int lafse3_get_params(const lafse3_ctx *ctx, lafse3_params *p);

/* Pre-allocate device workspace for launches of up to `n_instances` NLP instances so that later calls
 * with at most that many instances do no allocation (required before hipGraph capture).  A solve of B
 * instances needs B instances; sol_gradient needs 9*B.  The solver kernel is persistent (one wave per
 * SIMD slot pulling instances from a queue), so the workspace held is min(n_instances, slots) slots of
 * lafse3_workspace_bytes_per_instance() bytes, slots = CUs x 4 (1024 on MI355X). */
int lafse3_reserve(lafse3_ctx *ctx, int64_t n_instances);
/* Bytes of device workspace one NLP instance uses. */
int64_t lafse3_workspace_bytes_per_instance(void);

/* A HIP stream with a hardware queue of its own (every CU enabled), for launches of several contexts that are meant
 * to run concurrently.  HIP maps ordinary streams onto a small pool of hardware queues (GPU_MAX_HW_QUEUES, 4 by
 * default) by the process's stream history, and two streams that share a queue run their kernels one after the
 * other (the configs[4] episode groups then ran at 2/3 of the rate: profiles/r05_moving_trace.log).  Not a
 * reference entry point (serving plumbing).  device < 0: the caller's current device. */
int lafse3_stream_create(int device, void **stream);
int lafse3_stream_destroy(void *stream);

/* Batched OCSys.ocSolver (quad_OC.py:104-212) with the traversal cost of quad_model.py:200-213:
 *   ini_state B x 13, goal B x 3, p_tra B x 3, a_tra B x 3 (the 'tra_ang' vector of Rd2Rp,
 *   quad_policy.py:10-13, float64), t B (traversal time, used as given), u_last B x 4 or NULL (=0).
 * Outputs (each nullable): x B x (N+1) x 13 (state_traj_opt), u B x N x 4 (control_traj_opt),
 *   lam B x N x 13 (costate_traj_opt = IPOPT lam_g), cost B (sol['f']), status B, iters B. */
int lafse3_ocp_solve(lafse3_ctx *ctx, int64_t B, const double *ini_state, const double *goal,
                     const double *p_tra, const double *a_tra, const double *t, const double *u_last,
                     double *x, double *u, double *lam, double *cost, int32_t *status, int32_t *iters,
                     void *stream);

/* fp32 twin of lafse3_ocp_solve: the same arguments as float32 device buffers.  Inputs are
 * widened to fp64 and outputs rounded to fp32 on the device; the NLP itself is solved in fp64 (IPOPT's
 * 1e-8 tolerance, quad_OC.py:172, is below float32 resolution). */
int lafse3_ocp_solve_f32(lafse3_ctx *ctx, int64_t B, const float *ini_state, const float *goal,
                         const float *p_tra, const float *a_tra, const float *t, const float *u_last,
                         float *x, float *u, float *lam, float *cost, int32_t *status, int32_t *iters,
                         void *stream);

/* Batched run_quad.objective (quad_policy.py:67-91): t is rounded to one decimal (round(t,1) on a
 * float64), the NLP is solved, the rotor tracks (quad_model.py:239-276) are scored against the gate
 * gate12 B x 12 (4 corners, solid_geometry.obstacle) and the goal.  reward B, status B (nullable). */
int lafse3_objective(lafse3_ctx *ctx, int64_t B, const double *ini_state, const double *goal,
                     const double *gate12, const double *p_tra, const double *a_tra, const double *t,
                     const double *u_last, double *reward, int32_t *status, void *stream);

/* Batched run_quad.sol_gradient (quad_policy.py:94-112) on DNN outputs as emitted by torch:
 *   dnn_out B x 7 float32 = [p_tra(3), tra_ang(3), t].  9 NLP solves per sample (nominal, +1e-3 on
 *   each of the 6 pose variables, t-0.1, t+0.1), reference dtype quirks reproduced.
 *   u_last B x 4 or NULL (passed to the 6 perturbed solves only, as the reference does).
 * out8 B x 8 = [-drdx,-drdy,-drdz,-drda,-drdb,-drdc,-drdt, j]; rewards9 B x 9 and status9 B x 9
 * (nullable) expose the 9 rewards / solver statuses. */
int lafse3_sol_gradient(lafse3_ctx *ctx, int64_t B, const double *ini_state, const double *goal,
                        const double *gate12, const float *dnn_out, const double *u_last, double *out8,
                        double *rewards9, int32_t *status9, void *stream);

/* Batched run_quad.get_input (quad_policy.py:202-211): one NLP solve per sample on float32 DNN
 * outputs (t used unrounded), returns the first control u0 B x 4 and optionally the state
 * trajectory x B x (N+1) x 13 (nn_train_2.py:37-39 reads it). */
int lafse3_get_input(lafse3_ctx *ctx, int64_t B, const double *ini_state, const double *goal,
                     const double *u_last, const float *dnn_out, double *u0, double *x, int32_t *status,
                     void *stream);

/* Reward of given state trajectories x B x (N+1) x 13 (the scoring half of run_quad.objective,
 * quad_policy.py:78-91: rotor tips quad_model.py:239-276, obstacle.collis_det solid_geometry.py:104-168,
 * goal path term over rows N-4..N-1).  reward B.  Not a solver launch: the timing, counters and device error
 * word of the most recent solver launch (lafse3_last_kernel_ms / _last_counters / _check_device) are kept. */
int lafse3_reward(lafse3_ctx *ctx, int64_t B, const double *x, const double *goal, const double *gate12,
                  double *reward, void *stream);

/* Traversal time of the moving-gate loop for B episodes: quad_moving.py:29-57 (solver) -- the fixed point
 * t1 += (t2 - t1) / 2 of DNN2's time output on the gate advanced by velo t1 and pitched by w t1 (main.py:90-94
 * inputs), from t1 = |centroid - r| / 3 until |t2 - t1| <= 0.001 (at most 200 updates).  state B x 13, final_point
 * B x 3, gate12 B x 12 (4 corners), velo B x 3 (gate velocity of this plant step); dnn2_weights: the trained
 * DNN2 (18-128-128-7, nn3_1.pth) packed as l1.weight (128 x 18), l1.bias, l2.weight (128 x 128, row-major), l2.bias,
 * row 6 of l3.weight, l3.bias[6] (lafse3_dnn2_weight_count() floats, float32 as the reference evaluates it;
 * 16-byte aligned).
 * t_out B, iters B (updates taken; nullable). */
int lafse3_traversal_time(lafse3_ctx *ctx, int64_t B, const double *state, const double *final_point,
                          const double *gate12, const double *velo, double w, const float *dnn2_weights,
                          double *t_out, int32_t *iters, void *stream);
int lafse3_dnn2_weight_count(void);

/* Time (ms, HIP events on `stream`) of the most recent solver-kernel launch on this context (lafse3_reward
 * launches are not solver launches). */
float lafse3_last_kernel_ms(const lafse3_ctx *ctx);
/* Sum over the last launch of per-instance IPM iterations, Riccati sweeps and line-search trials
 * (written by the kernel; read back synchronously). counters[3].  Returns LAFSE3_EDEVICE (counters still
 * filled) while the device error word is set, i.e. when a solver launch since the last lafse3_check_device
 * raised it (not necessarily the last launch); lafse3_check_device reports and clears it. */
int lafse3_last_counters(lafse3_ctx *ctx, int64_t counters[3]);
/* Wait for the most recent solver launch on this context and return LAFSE3_EDEVICE (message via
 * lafse3_last_error) when a solver launch since the last such report raised the device error word: a
 * sol_gradient probe task whose queue entry never landed (its rewards9/status9 slot then holds NaN / status 7).
 * Launches do not clear the word; this call does, after reporting it.  0 otherwise. */
int lafse3_check_device(lafse3_ctx *ctx);
/* Restoration-phase counts of the last launch, summed over its NLP instances: counters[0] entries into the
 * restoration phase, counters[1] returns to the original problem (entries - returns ended the solve with
 * status 2, 4, 6, 8 or 9).  Read back synchronously; EDEVICE as lafse3_last_counters. */
int lafse3_last_resto_counters(lafse3_ctx *ctx, int64_t counters[2]);
/* Debug: subsequent launches write, per instance and per IPM iteration (< iters), 16 doubles
 * [mu, E0, theta, phi, gradphi.d, alpha_max, alpha_z, alpha, delta_w, accepted, filter_size, sweeps,
 *  refinement ratio 0/1/2, refinement count] to the device buffer buf (instances x iters x 16).
 * buf = NULL disables. */
int lafse3_debug_trace(lafse3_ctx *ctx, double *buf, int iters);
/* Debug: dump the Newton step [dx (51x13) | du (50x4) | lam+ (50x13)] of IPM iteration `it`
 * (before or after iterative refinement) into buf (instances x 1513).  buf = NULL disables. */
int lafse3_debug_dump(lafse3_ctx *ctx, double *buf, int it, int after_refine);
/* Debug: per-instance record of 32 x uint64 into buf (instances x 32).  The timer build (-DLAFSE3_PHASE_TIMERS)
 * fills columns 0..15 and 24..31, every build the placement record 16..23: 12 phase timers in s_memtime cycles (init, errors, table, backward, forward, adjoint, residual, refine-backward,
 * line search, accept, reward, other), 4 backward-sweep stage-phase timers, then the placement record: start and
 * end s_memrealtime (100 MHz), HW_ID and XCC_ID of the wave, then iterations, sweeps, status, trials; then 8
 * wait-probe sums (cycles spent in the factorisation stage's vector-memory waits, the last one the probes' own
 * cost). */
int lafse3_debug_timers(lafse3_ctx *ctx, uint64_t *buf);
/* Per-instance IPM iteration counts of subsequent launches into buf (int32, one per NLP instance: B for
 * ocp_solve / objective / get_input, B x 9 for sol_gradient in the rewards9 slot order; entry points that take
 * their own iters argument use that).  One store per instance; bench.py reads its percentiles.  capacity = the
 * entries buf holds: a later launch that would write more fails with LAFSE3_EINVAL.  NULL disables. */
int lafse3_record_iters(lafse3_ctx *ctx, int32_t *buf, int64_t capacity);
/* Debug (tests of the probe-queue guard): in later sol_gradient launches the queue entry of sample `sample`'s
 * probe solves is reserved but never written, so those probes are lost and the device error word is raised.
 * -1 disables. */
int lafse3_debug_drop_push(lafse3_ctx *ctx, int64_t sample);
const char *lafse3_last_error(void);
const char *lafse3_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LAFSE3_H */
