/*
 * rcbf_hip.h -- C-ABI of librcbf_hip.so, the MI355X (gfx950) batched safe-env
 * step of SAC-RCBF: control-affine dynamics + RCBF safety-layer QP.
 *
 * Every entry point replaces one reference interface (paths relative to the
 * reference repo yemam3/SAC-RCBF); the Python mirror in
 * sac-rcbf_amd/rcbf_amd/ binds them through ctypes.
 *
 * Conventions
 *   - All array arguments are CALLER-OWNED DEVICE pointers (PyTorch allocates;
 *     the library never allocates on the hot path).  Layouts are the
 *     reference's row-major tensors: x (B, n_s), u (B, n_u), G (B, m, n) ...
 *   - `stream` is the HIP stream to launch on (torch's current stream);
 *     every call is asynchronous, stateless and re-entrant (no globals), so
 *     one process per GPU or several streams are safe, and calls can be
 *     captured into a hipGraph.
 *   - Return value: 0 on success, otherwise a hipError_t value or one of the
 *     RCBF_E_* argument errors below.  Nothing throws across the ABI.
 *   - Per-QP solver status is written to device arrays (status_out) and
 *     OR-ed into an optional device word (fail_flag, bit (1<<status)) so the
 *     host can raise the reference's Exception('QP Failed to solve')
 *     (rcbf_sac/diff_cbf_qp.py:141-143) after a single 4-byte read.
 *   - Nullable pointers are marked [nullable].
 */
#ifndef RCBF_HIP_H
#define RCBF_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RCBF_ABI_VERSION 12

/* dynamics modes: rcbf_sac/dynamics.py:22-23 DYNAMICS_MODE */
#define RCBF_MODE_SIMULATED_CARS 0
#define RCBF_MODE_UNICYCLE 1

/* constraint formulations */
#define RCBF_FORM_DIFF 0    /* CBFQPLayer, rcbf_sac/diff_cbf_qp.py (fp32 rows, fp64 QP)  */
#define RCBF_FORM_CASCADE 1 /* CascadeCBFLayer, rcbf_sac/cbf_qp.py (fp64 rows, fp64 QP) */

/* QP solvers */
#define RCBF_SOLVER_ACTIVE_SET 0 /* exact, fp64: KKT enumeration (n=2) / Goldfarb-Idnani (n=3)          */
#define RCBF_SOLVER_PDIPM 1      /* primal-dual interior point, fp64 (qpth's algorithm family) + polish */
#define RCBF_SOLVER_GI 2         /* Goldfarb-Idnani dual active set for every n (quadprog's algorithm) */

/* per-QP status codes */
#define RCBF_QP_OK 0
#define RCBF_QP_MAX_ITER 1
#define RCBF_QP_INFEASIBLE 2
#define RCBF_QP_NONFINITE 3

/* argument errors (returned instead of a hipError_t) */
#define RCBF_E_BAD_MODE 1001
#define RCBF_E_BAD_SHAPE 1002
#define RCBF_E_NULL 1003
#define RCBF_E_HSA 1004     /* an HSA runtime call failed, or the AQL queue reported an error */
#define RCBF_E_TIMEOUT 1005 /* rcbf_aql_run: the dispatches did not complete in time */
#define RCBF_E_GP_HANDOFF 1006 /* rcbf_gp_workspace_check: a GEMV call found a non-zero arrival counter */

#define RCBF_MAX_HAZARDS 8

/* Layer + env constants.  Mirrors the ctor arguments of CBFQPLayer
 * (diff_cbf_qp.py:12-42) / CascadeCBFLayer (cbf_qp.py:7-27) and the env
 * attributes they read (kp, k_brake, safe_action_space, hazards_*).  */
typedef struct rcbf_params {
    int32_t mode;        /* RCBF_MODE_*                                   */
    int32_t formulation; /* RCBF_FORM_*                                   */
    int32_t num_hazards; /* unicycle: len(env.hazards_locations) <= 8     */
    int32_t solver;      /* RCBF_SOLVER_*                                  */
    int32_t max_iter;    /* solver iteration cap (0 -> default)           */
    int32_t _pad;
    double gamma_b;      /* gamma of the barrier certificate              */
    double k_d;          /* confidence multiplier (Cascade unicycle only) */
    double l_p;          /* look-ahead distance (unicycle)                */
    double kp, k_brake;  /* cars gains (simulated_cars_env.py:25-26)      */
    double u_min[2], u_max[2]; /* env.safe_action_space.low/high          */
    double hazards_radius;
    double hazards_xy[2 * RCBF_MAX_HAZARDS];
    double eps;          /* PDIPM stopping tolerance (qpth eps, default 1e-4 -> we use 1e-10) */
} rcbf_params;

/* ---------------------------------------------------------------------- */
/* CBF-QP layer                                                            */
/* ---------------------------------------------------------------------- */

/* CBFQPLayer.get_cbf_qp_constraints (diff_cbf_qp.py:146-379), fp32.
 * x, mu, sigma (B, n_s); u_rl (B, n_u).  mu/sigma [nullable] -> the
 * DynamicsModel prior (dynamics.py:381-384: mean 0, sigma MAX_STD).
 * Outputs P (B,n,n), q (B,n), G (B,m,n), h (B,m) with n = n_u+1 and
 * m = num_cbfs + 2 n_u, row order as the reference. */
int rcbf_build(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl,
               const float* mu, const float* sigma, float* P_out, float* q_out,
               float* G_out, float* h_out, hipStream_t stream);

/* CascadeCBFLayer.get_cbf_qp_constraints (cbf_qp.py:55-240), fp64, batched. */
int rcbf_build_f64(const rcbf_params* prm, int64_t B, const double* x, const double* u_nom,
                   const double* mu, const double* sigma, double* P_out, double* q_out,
                   double* G_out, double* h_out, hipStream_t stream);

/* CBFQPLayer.solve_qp + cbf_layer (diff_cbf_qp.py:81-144): optional row
 * normalisation (normalize=1: rows of [G h] divided by their max-abs entry,
 * :103-106), then  min 1/2 z'Pz + q'z  s.t.  Gz <= h  in fp64 for a general
 * SPD P (n <= 3, m <= 16).  z_out fp32 (the reference's .float()).
 * lam_out [nullable] (B,m) fp64 multipliers; status_out [nullable] (B,);
 * fail_flag [nullable] one device int32, OR-ed with (1<<status) on failure. */
int rcbf_qp_solve(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P,
                  const float* q, const float* G, const float* h, int32_t normalize,
                  float* z_out, double* lam_out, int32_t* status_out, int32_t* fail_flag,
                  hipStream_t stream);

/* CascadeCBFLayer.solve_qp (cbf_qp.py:242-286, quadprog on the row-normalised
 * problem): rcbf_qp_solve with fp64 inputs and an fp64 solution z_out (B,n). */
int rcbf_qp_solve_f64(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const double* P,
                      const double* q, const double* G, const double* h, int32_t normalize,
                      double* z_out, double* lam_out, int32_t* status_out, int32_t* fail_flag,
                      hipStream_t stream);

/* Backward of rcbf_qp_solve: CBFQPLayer.cbf_layer / solve_qp under autograd
 * (diff_cbf_qp.py:81-144 -> qpth QPFunction.backward, diff_cbf_qp.py:139).
 * Recomputes the exact forward in-kernel, then the implicit-KKT adjoint on
 * the active set: grad_q = dz, grad_P = (dz z' + z dz')/2,
 * grad_G = eta z' + lam dz', grad_h = -eta, pulled back through the row
 * normaliser when normalize=1 (:103-106, torch.max/abs autograd rules).
 * grad_z (B,n) in; grad_P (B,n,n), grad_q (B,n), grad_G (B,m,n),
 * grad_h (B,m) out, each [nullable]; q [nullable] = 0. */
int rcbf_qp_backward(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P,
                     const float* q, const float* G, const float* h, int32_t normalize,
                     const float* grad_z, float* grad_P, float* grad_q, float* grad_G,
                     float* grad_h, hipStream_t stream);

/* The forward/backward pair with the forward's solution saved, as qpth's
 * QPFunction keeps zhats / lams for its backward (diff_cbf_qp.py:139; the
 * autograd surface of solve_qp / cbf_layer uses this pair).
 * rcbf_qp_solve_saved: rcbf_qp_solve that also writes the fp64 solution
 * z64_saved (B,n).  rcbf_qp_backward_saved: rcbf_qp_backward that starts from
 * z64_saved instead of re-solving: for a diagonal P and q = 0 the tight rows,
 * multipliers and adjoint come from one factorisation on them; a QP whose
 * KKT certificate fails there (or a full P / nonzero q) re-solves exactly,
 * as rcbf_qp_backward does.  z64_saved must come from rcbf_qp_solve_saved on
 * the same inputs. */
int rcbf_qp_solve_saved(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P,
                        const float* q, const float* G, const float* h, int32_t normalize,
                        float* z_out, double* z64_saved, int32_t* status_out, int32_t* fail_flag,
                        hipStream_t stream);
int rcbf_qp_backward_saved(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P,
                           const float* q, const float* G, const float* h, int32_t normalize,
                           const double* z64_saved, const float* grad_z, float* grad_P,
                           float* grad_q, float* grad_G, float* grad_h, hipStream_t stream);

/* CBFQPLayer.get_safe_action (diff_cbf_qp.py:44-79), fused in one kernel:
 * build -> normalise -> fp64 QP -> .float() -> clamp(u_rl + u_qp, u_min, u_max).
 * mu/sigma [nullable] -> prior.  u_out (B, n_u) fp32. */
int rcbf_safe_action(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl,
                     const float* mu, const float* sigma, float* u_out, int32_t* status_out,
                     int32_t* fail_flag, hipStream_t stream);

/* Backward of rcbf_safe_action w.r.t. u_rl (the only input the reference's
 * autograd reaches, sac_cbf.py:147-158): implicit-KKT derivative of the QP on
 * its active set (what qpth's QPFunction.backward approximates), through the
 * row normaliser and the clamp.  Recomputes the forward in-kernel (no saved
 * tensors).  grad_u (B,n_u) in, grad_u_rl (B,n_u) out. */
int rcbf_safe_action_backward(const rcbf_params* prm, int64_t B, const float* x,
                              const float* u_rl, const float* mu, const float* sigma,
                              const float* grad_u, float* grad_u_rl, hipStream_t stream);

/* RCBF_SAC.get_safe_action (sac_cbf.py:218-238) with the prior disturbance
 * model, as the SAC update calls it on replay batches (sac_cbf.py:133,149):
 * DynamicsModel.get_state (dynamics.py:190-232) from the fp32 observation
 * obs (B,n_o) in-kernel, then exactly rcbf_safe_action.  mu/sigma (B,n_s)
 * [nullable: the MAX_STD prior of predict_disturbance, dynamics.py:381-384]. */
int rcbf_obs_safe_action(const rcbf_params* prm, int64_t B, const float* obs,
                         const float* u_rl, const float* mu, const float* sigma,
                         float* u_out, int32_t* status_out, int32_t* fail_flag,
                         hipStream_t stream);

/* Backward of rcbf_obs_safe_action w.r.t. u_rl (the policy's action; obs,
 * mean and sigma are detached in the reference, dynamics.py:211,362). */
int rcbf_obs_safe_action_backward(const rcbf_params* prm, int64_t B, const float* obs,
                                  const float* u_rl, const float* mu, const float* sigma,
                                  const float* grad_u, float* grad_u_rl, hipStream_t stream);

/* rcbf_safe_action / rcbf_obs_safe_action that also keep what their
 * backward needs, as qpth's QPFunction keeps its solution for the backward
 * (the forward the SAC update differentiates, sac_cbf.py:147-158): u_out
 * exactly as the plain forward, plus jac_out (B, n_u, n_u) f64 =
 * d final / d u_rl on the exact active set, through the normaliser, with the
 * clamp folded in (a saturated action's row holds RCBF_JAC_NO_GRAD, a NaN
 * with its own payload, "no gradient"; any other NaN came from the solve and
 * propagates).  rcbf_safe_action_apply_jac is then the whole backward:
 * grad_u_rl = grad_u . jac over the rows not marked RCBF_JAC_NO_GRAD, bit for
 * bit what rcbf_[obs_]safe_action_backward computes, without the second
 * solve. */
#define RCBF_JAC_NO_GRAD 0x7FFCD0C0FFEE0000ULL
int rcbf_safe_action_jac(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl,
                         const float* mu, const float* sigma, float* u_out, double* jac_out,
                         int32_t* status_out, int32_t* fail_flag, hipStream_t stream);
int rcbf_obs_safe_action_jac(const rcbf_params* prm, int64_t B, const float* obs,
                             const float* u_rl, const float* mu, const float* sigma, float* u_out,
                             double* jac_out, int32_t* status_out, int32_t* fail_flag,
                             hipStream_t stream);
int rcbf_safe_action_apply_jac(int64_t B, int32_t n_u, const double* jac, const float* grad_u,
                               float* grad_u_rl, hipStream_t stream);

/* CascadeCBFLayer.get_u_safe (cbf_qp.py:29-53), fp64 batched: build ->
 * normalise -> exact QP.  Returns u_qp only (caller adds u_nom, no clamp);
 * eps_out [nullable] (B,) f64 receives the slack epsilon, the QP solution's
 * last component (sol[0][-1], which the reference checks against 0.1 at
 * cbf_qp.py:283-284). */
int rcbf_cascade_u_safe(const rcbf_params* prm, int64_t B, const double* u_nom,
                        const double* x, const double* mu, const double* sigma,
                        double* u_safe_out, int32_t* status_out, int32_t* fail_flag,
                        double* eps_out, hipStream_t stream);

/* rcbf_cascade_u_safe for B <= 256 samples in ONE workgroup that ends by
 * storing `seq` into done_word (pinned host memory, system scope); the call
 * returns when it reads `seq`.  Every array may be pinned host memory
 * (rcbf_host_alloc: the kernel reads and writes it in place) or device
 * memory, so the reference's single-sample get_u_safe of its per-step loop
 * (envs/simulated_cars_env.py:213, cbf_qp.py:29-53) costs no copy and no
 * stream synchronisation.  status_out, eps_out, mu, sigma [nullable]. */
int rcbf_cascade_u_safe_sync(const rcbf_params* prm, int64_t B, const double* u_nom,
                             const double* x, const double* mu, const double* sigma,
                             double* u_safe_out, int32_t* status_out, double* eps_out,
                             uint32_t* done_word, uint32_t seq, hipStream_t stream);

/* ---------------------------------------------------------------------- */
/* GP disturbance posterior                              */
/* ---------------------------------------------------------------------- */
/* The fitted disturbance model of DynamicsModel (dynamics.py:296-340): one
 * exact GP per state dimension i (ScaleKernel(RBF) + Gaussian likelihood,
 * gp_model.py:12-27) on shared normalised training inputs.  Built on the
 * host after each fit (rcbf_amd.gp); all arrays are device memory. */
#define RCBF_GP_RT_UPPER 1

typedef struct rcbf_gp_model {
    int32_t n_s;     /* GPs = state dims = input dims (3 or 10)                 */
    int32_t N;       /* training points                                         */
    int32_t N_pad;   /* N rounded up to a multiple of 32 (padding rows: Rt = 0)  */
    int32_t r;       /* rank of the variance factor (r = N: exact posterior)     */
    int32_t C_pad;   /* columns of Rt per GP: multiple of 128, >= r + 1          */
    int32_t flags;   /* RCBF_GP_RT_UPPER: logical column j < r of Rt is zero below
                        row j (R = L^-T of the exact Cholesky factor), so column
                        block cb reads only training rows < 128 (cb + 1)          */
    const float* xt;       /* (n_s, N_pad, n_s): train_x / (std + 1e-8) / (sqrt2 l_i) */
    const float* tn2;      /* (n_s, N_pad): squared norms of the xt rows             */
    const float* Rt;       /* (n_s, N_pad, C_pad): [R_i | alpha_i | 0], R R^T = (K+nI)^-1;
                              within each 128-column block, physical column 4 l + c
                              holds logical column 32 c + l (16-B loads per lane)   */
    const double* x_std;   /* (n_s,): train_x std; queries are x / x_std (no +1e-8,
                              dynamics.py:376)                                       */
    const float* inv_sl;   /* (n_s,): 1 / (sqrt(2) l_i)                              */
    const float* outscale; /* (n_s,): s_i                                            */
    const float* noise;    /* (n_s,): likelihood noise n_i                           */
    const float* y_scale;  /* (n_s,): train_y std + 1e-8 (dynamics.py:379-380)      */
} rcbf_gp_model;

/* Floats of workspace rcbf_gp_predict needs for B queries.  Its first words
 * are the arrival counters of the one-launch GEMV path (B <= 8): a workspace
 * must be ZERO-FILLED before its first use (e.g. torch.zeros); every call
 * leaves those words zero again.  One workspace per concurrent call (per
 * stream); rcbf_gp_workspace_check detects a violation after the fact. */
int64_t rcbf_gp_workspace_floats(const rcbf_gp_model* m, int64_t B);

/* Zero the workspace's counter words (hipMemsetAsync on `stream`): the
 * initialisation a new workspace needs before its first rcbf_gp_predict. */
int rcbf_gp_workspace_init(const rcbf_gp_model* m, float* workspace, hipStream_t stream);

/* SYNCHRONOUS check of the one-launch GEMV hand-off (waits for `stream`): a
 * GEMV workgroup that draws an arrival ticket past its block's (or GP's)
 * arrival count proves the counter was not zero when its call started -- the
 * workspace was not zero-filled, a call was aborted part-way, or two calls
 * shared the workspace at once -- and sets the workspace's fail word; the
 * outputs of such a call are not valid.  A counter that started off by less
 * than its arrival count lets an early workgroup take the "last" ticket; such a
 * call leaves its counter non-zero once the stream has drained, which the check
 * also reads as a failure.  Returns RCBF_E_GP_HANDOFF if the word is set or any
 * counter is non-zero, after zeroing every counter and the word (the next call
 * is clean); 0 otherwise. */
int rcbf_gp_workspace_check(const rcbf_gp_model* m, float* workspace, hipStream_t stream);

/* DynamicsModel.predict_disturbance(test_x) with fitted GPs (dynamics.py:
 * 342-390, gp_model.py:86-114): x (B, n_s) f32 states -> mean (B, n_s) and
 * std (B, n_s) f32, std = sqrt(latent variance + noise) (the likelihood's
 * predictive variance), both rescaled by y_scale.  Exact GP posterior when
 * r = N; gpytorch's fast_pred_var (LOVE, gp_model.py:97-99) above 800
 * training points is a rank-100 Lanczos R built by the host.  B <= 8: ONE
 * launch (a streaming GEMV whose last workgroups finish the posterior); B > 8:
 * the k(x, X) [R | alpha] GEMM on the fp32 MFMA (split-K + combine when the
 * grid is small), then a per-row finish. */
int rcbf_gp_predict(const rcbf_gp_model* m, int64_t B, const float* x, float* mean_out,
                    float* std_out, float* workspace, hipStream_t stream);

/* RCBF_SAC.get_safe_action of ONE observation with the fitted GP (sac_cbf.py:
 * 218-238 as main.py:93 calls it, through select_action, every env step) in
 * ONE launch: get_state(obs) (dynamics.py:190-232) formed in every workgroup,
 * the GP posterior of rcbf_gp_predict's B <= 8 GEMV on it (dynamics.py:342-
 * 390), and, in the last workgroup to finish a GP, the one-launch safe action
 * on the posterior (diff_cbf_qp.py:44-79: rows, normalisation, exact QP,
 * clamp) -- the arithmetic of rcbf_state_from_obs -> rcbf_gp_predict ->
 * rcbf_obs_safe_action, so the action is bit-equal to those three launches.
 * B must be 1; prm: the layer (solver RCBF_SOLVER_ACTIVE_SET, mode matching
 * m->n_s).  obs (1, n_o), u_rl (1, n_u) f32 device; mean_out / std_out
 * [nullable] (1, n_s) the posterior; u_out [nullable] (1, n_u) f32 device;
 * u_host [nullable] (1, n_u) f32 in pinned host memory (rcbf_host_alloc);
 * done_word [nullable] a pinned host word: when given, the kernel stores `seq`
 * into it (system scope) after the action, and the call RETURNS WHEN IT READS
 * `seq` -- the action is then on the host, with no copy or stream
 * synchronisation (as rcbf_env_step_sync).  The workspace is the GP's
 * (rcbf_gp_workspace_floats(m, 1), zero-filled once).  RCBF_E_BAD_MODE for
 * another solver; RCBF_E_BAD_SHAPE for B != 1 or a model of another width;
 * RCBF_E_GP_HANDOFF (done_word given) when the kernel completed without
 * publishing: a hand-off counter was not zero at the start, so no result was
 * formed (rcbf_gp_workspace_check then reports and zeroes the counters). */
int rcbf_gp_obs_safe_action(const rcbf_params* prm, const rcbf_gp_model* m, int64_t B, const float* obs,
                            const float* u_rl, float* mean_out, float* std_out, float* u_out, float* u_host,
                            uint32_t* done_word, uint32_t seq, int32_t* status_out, int32_t* fail_flag,
                            float* workspace, hipStream_t stream);

/* rcbf_gp_predict that also (or only) writes the COLUMN layout the fused
 * step reads (rcbf_safe_step_cols): mean_cols / std_cols (n_cols, B) f32 of
 * the output dimensions cols[0..n_cols) (a host array, n_cols <= 10), e.g.
 * cars std columns {5, 7, 9}.  mean_out / std_out (B, n_s) and the column
 * outputs are each nullable (at least one output). */
int rcbf_gp_predict_cols(const rcbf_gp_model* m, int64_t B, const float* x, float* mean_out,
                         float* std_out, const int32_t* cols, int32_t n_cols, float* mean_cols,
                         float* std_cols, float* workspace, hipStream_t stream);

/* ---------------------------------------------------------------------- */
/* Model-based rollouts and the device replay buffer  */
/* ---------------------------------------------------------------------- */
/* One k-step of generate_model_rollouts (rcbf_sac/generate_rollouts.py:24-77)
 * on B replay transitions, fp64: state = get_state(obs); mu = model prior
 * x + dt (f + g a) + dt * mean; next_state = mu + dt * std * z; next_obs =
 * get_obs(next_state) (+ compass, exp(-dist) for the unicycle); reward, mask
 * (= not done), next_t = t + dt.  obs (B,n_o) f64, act (B,n_u) f64, t (B,) f64
 * [nullable for the unicycle]; mean/std (B,n_s) f32 [nullable: the MAX_STD
 * prior]; z (B,n_s) f64 N(0,1) draws [nullable: Philox4x32-10 keyed by
 * (seed, row, counter)]. */
int rcbf_model_step(const rcbf_params* prm, int64_t B, const double* obs, const double* act,
                    const double* t, const float* mean, const float* std, const double* z,
                    uint64_t seed, uint64_t counter, double* next_obs, double* reward,
                    double* mask, double* next_t, hipStream_t stream);

/* DynamicsModel.predict_next_state (rcbf_sac/dynamics.py:60-105) on device
 * rows, fp64: next_x = x + dt (f(x) + g(x) u) (+ dt * mean when use_gps),
 * std_out = dt * std (zeros when !use_gps), next_t = t + dt [nullable].
 * x (B,n_s) f64, act (B,n_u) f64, t (B,) f64 [nullable for the unicycle];
 * mean/std (B,n_s) f32, the GP posterior [nullable: the zero-mean MAX_STD
 * prior, dynamics.py:381-384]. */
int rcbf_predict_next_state(const rcbf_params* prm, int64_t B, const double* x, const double* act,
                            const double* t, const float* mean, const float* std, int32_t use_gps,
                            double* next_x, double* std_out, double* next_t, hipStream_t stream);

/* DynamicsModel.get_state (rcbf_sac/dynamics.py:190-232) on fp32
 * observation rows, one launch: obs (B, n_o) f32 -> state (B, n_s) f32 with
 * the reference's arithmetic (to numpy fp64, cars x100 / x30, unicycle
 * arctan2(sin, cos), back to fp32) -- the state that rcbf_obs_safe_action
 * builds in-kernel, for the GP query of RCBF_SAC.get_safe_action
 * (sac_cbf.py:233-236). */
int rcbf_state_from_obs(const rcbf_params* prm, int64_t B, const float* obs, float* state_out,
                        hipStream_t stream);

/* ReplayMemory.batch_push (replay_memory.py:23-29) as one launch: n records
 * of W f64 (state, action, reward, next_state, mask, t, next_t packed) into
 * the ring of `cap` records starting at record `pos` (wrapping). */
int rcbf_ring_scatter_f64(double* ring, int64_t cap, int64_t W, int64_t pos,
                          const double* src, int64_t n, hipStream_t stream);

/* ReplayMemory.sample (replay_memory.py:31-35) gather: dst[r] = ring[idx[r]]. */
int rcbf_gather_rows_f64(double* dst, const double* ring, int64_t W, const int64_t* idx,
                         int64_t n, hipStream_t stream);

/* ---------------------------------------------------------------------- */
/* Environments (batched, device-resident, fp64 state like the numpy envs) */
/* ---------------------------------------------------------------------- */
/* Per-env state, COMPONENT-PAIR-MAJOR:  x (n_s * B) f64, 16-byte aligned;
 * components (2p, 2p+1) of env i at x[2*(p*B + i)] and x[2*(p*B + i) + 1]
 * (one (B, 2) block per pair, so a lane moves 16 B per pair and a wavefront
 * 1 KiB contiguous), and for odd n_s the last component at x[(n_s-1)*B + i].
 * x = env_i.state;  aux (B,) f64 = env.t (cars) or env.last_goal_dist
 * (unicycle);  step (B,) i32 = env.episode_step;  episode (B,) u32 = reset
 * counter keying the per-env counter-based RNG (read/written only on reset).
 * Observations are row-major (B, n_o), the policy's input layout, 8-byte
 * aligned.  (For B = 1 the state layout is the state row itself.)
 * A misaligned x or obs returns RCBF_E_BAD_SHAPE.  */

/* SimulatedCarsEnv.reset (simulated_cars_env.py:108-125) / UnicycleEnv.reset
 * (unicycle_env.py:125-143) for the envs selected by mask [nullable: all].
 * noise [nullable] (B,) f64 injects the cars' N(0,0.5) velocity draw; when
 * null it comes from a Philox4x32-10 counter RNG keyed by (seed, env_offset + env
 * index, episode): env_offset is the global index of env 0 of this shard, so a
 * sharded run draws exactly what the unsharded run draws.
 * obs_out [nullable] (B, n_o) f32. */
int rcbf_env_reset(const rcbf_params* prm, int64_t B, const uint8_t* mask, const double* noise,
                   uint64_t seed, int64_t env_offset, double* x, double* aux, int32_t* step,
                   uint32_t* episode, float* obs_out, hipStream_t stream);

/* env.step(action) (simulated_cars_env.py:38-106, unicycle_env.py:46-111),
 * batched.  action (B, n_u), fp32 (action_f64 = 0) or fp64 (action_f64 = 1);
 * the cars reward is computed in the action's dtype like the reference.
 * Outputs: obs64_out [nullable] (B,n_o) f64, obs_out [nullable] (B,n_o) f32,
 * reward (B,) f64, cost (B,) f64, done (B,) u8, goal_met [nullable] (B,) u8.
 * auto_reset=1 resets finished envs in place (obs = post-reset obs). */
int rcbf_env_step(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step,
                  uint32_t* episode, const void* action, int32_t action_f64, double* obs64_out,
                  float* obs_out, double* reward, double* cost, uint8_t* done, uint8_t* goal_met,
                  int32_t auto_reset, uint64_t seed, int64_t env_offset, hipStream_t stream);

/* The reference's per-step gym call (env.step at main.py:95) for a small
 * batch that lives on the device but talks to the host: the action is READ
 * from host memory and obs64 / reward / cost / done / goal_met are WRITTEN
 * to host memory by the kernel itself (zero copy, both buffers from
 * rcbf_host_alloc).  One host call, no copy launches.  For B <= 256 the
 * kernel then stores a sequence number into a completion word in
 * packed_host, after a system-scope fence, and the call returns once the
 * word holds it (polling; the stream is asked every 4096 polls, so a failed
 * kernel returns its error); for larger B the call waits for the stream.
 * packed_host (W + 4 bytes, W = (B (8 (n_o + 2) + 2) + 7) & ~7) holds
 *   obs64 (B, n_o) f64 | reward (B,) f64 | cost (B,) f64 | done (B,) u8 | goal_met (B,) u8
 *   | pad to 8 B | completion word u32 at byte offset W.
 * action_host (B, n_u) f32 (action_f64 = 0) or f64 (action_f64 = 1).
 * Same arithmetic as rcbf_env_step. */
int rcbf_env_step_sync(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step,
                       uint32_t* episode, const void* action_host, int32_t action_f64, double* packed_host,
                       int32_t auto_reset, uint64_t seed, int64_t env_offset, hipStream_t stream);

/* Pinned, device-coherent host memory for rcbf_env_step_sync (set-up only,
 * never on the per-step path).  Returns hipError_t; *ptr = NULL on failure. */
int rcbf_host_alloc(int64_t bytes, void** ptr);
int rcbf_host_free(void* ptr);

/* The fused safe step -- the hot path measured by bench.py:
 *   obs32 = float(obs(x)); state = get_state(obs32) (dynamics.py:190-232);
 *   mean,sigma = prior or given; u = CBFQPLayer.get_safe_action(state, u_rl,
 *   mean, sigma); env.step(u) with optional auto-reset; obs32 of the new state.
 * All in one launch, one env per lane, env state read and written in place.
 * u_out (B,n_u) f32 safe action; reward/cost (B,) f32; done (B,) u8;
 * goal_met [nullable]; status_out [nullable]; fail_flag [nullable]. */
int rcbf_safe_step(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step,
                   uint32_t* episode, const float* u_rl, const float* mu, const float* sigma,
                   float* obs_out, float* u_out, float* reward, float* cost, uint8_t* done,
                   uint8_t* goal_met, int32_t* status_out, int32_t* fail_flag,
                   int32_t auto_reset, uint64_t seed, int64_t env_offset, hipStream_t stream);

/* rcbf_safe_step with the disturbance prediction in COLUMN layout: only the
 * entries the CBF rows read, one contiguous (B,) f32 column each, as
 * rcbf_gp_predict_cols writes them after a GP fit (dynamics.py:342-390
 * feeding diff_cbf_qp.py:241, 261, 299).  Cars: sigma_cols (3, B) =
 * sigma[:, 5], sigma[:, 7], sigma[:, 9]; mu_cols must be NULL (the cars rows
 * ignore the mean).  Unicycle: mu_cols, sigma_cols (3, B).  NULL -> the
 * prior, as in rcbf_safe_step.  Same results as rcbf_safe_step on the
 * (B, n_s) rows holding the same values; 12 B instead of whole 40-B rows per
 * cars env. */
int rcbf_safe_step_cols(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step,
                        uint32_t* episode, const float* u_rl, const float* mu_cols, const float* sigma_cols,
                        float* obs_out, float* u_out, float* reward, float* cost, uint8_t* done,
                        uint8_t* goal_met, int32_t* status_out, int32_t* fail_flag, int32_t auto_reset,
                        uint64_t seed, int64_t env_offset, hipStream_t stream);

/* K fused safe steps issued back to back from one host call: K launches of
 * the same kernel as rcbf_safe_step on `stream` (each step reads and writes
 * the env state in HBM; outputs are overwritten each step).  Step j reads the
 * policy actions u_rl_seq[j % n_u_rl], a HOST array of n_u_rl device
 * pointers, each (B, n_u) f32.  The batched training / warm-up loop
 * (main.py:47-110 with actions already on the device) without a Python
 * round trip or a graph launch per step.  Stops at the first failing launch
 * and returns its error. */
int rcbf_safe_step_seq(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux,
                       int32_t* step, uint32_t* episode, const float* const* u_rl_seq, int32_t n_u_rl,
                       const float* mu, const float* sigma, float* obs_out, float* u_out, float* reward,
                       float* cost, uint8_t* done, uint8_t* goal_met, int32_t* status_out,
                       int32_t* fail_flag, int32_t auto_reset, uint64_t seed, int64_t env_offset,
                       hipStream_t stream);

/* rcbf_safe_step_seq with the disturbance prediction in the column layout
 * of rcbf_safe_step_cols (same arguments and rules as that entry point). */
int rcbf_safe_step_seq_cols(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux,
                            int32_t* step, uint32_t* episode, const float* const* u_rl_seq, int32_t n_u_rl,
                            const float* mu_cols, const float* sigma_cols, float* obs_out, float* u_out,
                            float* reward, float* cost, uint8_t* done, uint8_t* goal_met,
                            int32_t* status_out, int32_t* fail_flag, int32_t auto_reset, uint64_t seed,
                            int64_t env_offset, hipStream_t stream);

/* MEASUREMENT entry point (bench.py's untraced kernel span; not a reference
 * interface): rcbf_safe_step (prior_cols = 0) or rcbf_safe_step_cols
 * (prior_cols = 1), the same instructions, plus per wavefront w (lanes
 * 64w..64w+63 of the launch, w < ceil(B / 64)) lane 0 writes the 100 MHz chip
 * clock (s_memrealtime) at the wave's start and after its own stores have
 * completed: span_out[4w], span_out[4w+1], and the shader clock (s_memtime)
 * at the same two points: span_out[4w+2], span_out[4w+3] (uint64, 16-B
 * aligned; delta(memtime) / delta(memrealtime) x 100 MHz = the clock).  The
 * launch's kernel span is max(end) - min(start) over its waves. */
int rcbf_safe_step_span(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step,
                        uint32_t* episode, const float* u_rl, const float* mu, const float* sigma,
                        int32_t prior_cols, float* obs_out, float* u_out, float* reward, float* cost,
                        uint8_t* done, uint8_t* goal_met, int32_t* status_out, int32_t* fail_flag,
                        int32_t auto_reset, uint64_t seed, int64_t env_offset, uint64_t* span_out,
                        hipStream_t stream);

/* K fused safe steps in ONE launch with the env state held in registers
 * (a pre-sampled u_rl (K, B, n_u), e.g. the reference's warm-up phase that
 * samples action_space uniformly, main.py:88-92).  Per-step outputs are
 * reduced per env: reward_sum, cost_sum (B,) f32, episodes finished (B,) i32.
 * obs_out [nullable] (B,n_o) f32 final observation. */
int rcbf_safe_rollout(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux,
                      int32_t* step, uint32_t* episode, const float* u_rl, float* obs_out,
                      float* reward_sum, float* cost_sum, int32_t* n_done, int32_t* fail_flag,
                      uint64_t seed, int64_t env_offset, hipStream_t stream);

/* ---------------------------------------------------------------------- */
/* The fused safe step on a user-mode AQL queue of the library's own
 * (csrc/rcbf_aql.hip).  Same kernels, same machine code as rcbf_safe_step --
 * the gfx950 code object of rcbf_env.o, unbundled at build time into
 * librcbf_steps.co -- dispatched as pre-built AQL packets instead of through
 * the HIP launch path, so K steps cost ~1 us of host time instead of a
 * hipGraph launch (~16-25 us host, ~17 us before the first kernel starts) or
 * K hipLaunchKernel calls (~5 us each).
 *
 * Replaces: env.step() of the batched env in the SAC loop (main.py:93-95 with
 * sac_cbf.py:218-238), K steps per call; like a gym step the call is
 * SYNCHRONOUS: rcbf_aql_run returns after the K steps have completed.  The
 * queue is not a HIP stream: the caller orders it against HIP work by
 * synchronising before the run (inputs written by HIP kernels must be
 * complete); HIP work issued after the run sees its results.
 *
 * rcbf_aql_open: device = HIP device ordinal; code_object [nullable] = path
 * of librcbf_steps.co (NULL: next to librcbf_hip.so); flags RCBF_AQL_PROFILE
 * enables per-dispatch timestamps (hsa_amd_profiling) on the queue.  One
 * producer thread per queue.
 * rcbf_aql_safe_step_plan: the arguments of rcbf_safe_step_seq (prior_cols =
 * 1: the column layout of rcbf_safe_step_cols) plus span_out [nullable] (the
 * measurement instantiation of rcbf_safe_step_span; step j writes its stamps
 * to span_out[4 ceil(B/64) j ...], K blocks of rcbf_safe_step_span's layout); the K
 * kernel-argument blocks are copied to device memory here (synchronous), so
 * the buffers must stay allocated while the plan exists.  flags
 * RCBF_AQL_PROFILE: a completion signal per dispatch, read back with
 * rcbf_aql_plan_times (start, end in ns of the HSA system clock per step);
 * RCBF_AQL_PROFILE_ENDS: on the first and last dispatch only (the others
 * read back as 0).
 * rcbf_aql_run: submit the K dispatches (barrier bit on each), ring the
 * doorbell once, busy-wait for completion; timeout_us 0 -> 10 s.  A plan
 * must not run after rcbf_aql_close of its queue (rcbf_aql_plan_free may
 * still be called then).
 * Returns RCBF_E_HSA / RCBF_E_TIMEOUT on a queue error or a timeout. */
#define RCBF_AQL_PROFILE 1
/* plan flags: memory-fence scopes (default: agent scope everywhere but the
 * last packet's release, which is system scope) */
#define RCBF_AQL_FIRST_ACQUIRE_SYSTEM 2 /* the first step acquires at system scope (inputs in host memory) */
#define RCBF_AQL_LAST_RELEASE_AGENT 4   /* the last step releases at agent scope */
#define RCBF_AQL_STUDY_MID_NOFENCE 8    /* STUDY ONLY: no fences between steps (not coherent across XCDs) */
#define RCBF_AQL_STUDY_MID_NOACQ 16     /* STUDY ONLY: no acquire between steps */
#define RCBF_AQL_STUDY_MID_NOREL 32     /* STUDY ONLY: no release between steps */
#define RCBF_AQL_PROFILE_ENDS 64        /* timestamps of the first and the last dispatch only */
#define RCBF_AQL_SAFE_STEP_KERNARG_BYTES 408 /* sizeof the k_safe_step argument block */
typedef struct rcbf_aql rcbf_aql;
typedef struct rcbf_aql_plan rcbf_aql_plan;
int rcbf_aql_open(int32_t device, const char* code_object, int32_t flags, rcbf_aql** out);
int rcbf_aql_close(rcbf_aql* q);
int rcbf_aql_kernel_count(const rcbf_aql* q);
int rcbf_aql_safe_step_plan(rcbf_aql* q, const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux,
                            int32_t* step, uint32_t* episode, const float* const* u_rl_seq, int32_t n_u_rl,
                            const float* mu, const float* sigma, int32_t prior_cols, float* obs_out, float* u_out,
                            float* reward, float* cost, uint8_t* done, uint8_t* goal_met, int32_t* status_out,
                            int32_t* fail_flag, int32_t auto_reset, uint64_t seed, int64_t env_offset,
                            uint64_t* span_out, int32_t flags, rcbf_aql_plan** out);
int rcbf_aql_run(rcbf_aql_plan* plan, uint64_t timeout_us);
int rcbf_aql_plan_times(const rcbf_aql_plan* plan, uint64_t* start_end_ns);
int rcbf_aql_plan_free(rcbf_aql_plan* plan);

/* ---------------------------------------------------------------------- */
const char* rcbf_version(void);
int32_t rcbf_abi_version(void);
/* sizeof(rcbf_params) as compiled, for binding checks (no GPU needed). */
int32_t rcbf_params_size(void);

#ifdef __cplusplus
}
#endif
#endif /* RCBF_HIP_H */
