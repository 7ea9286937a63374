// rcbf_env.hip -- device-resident environments and the fused safe step + C-ABI:
// rcbf_env_reset, rcbf_env_step, rcbf_env_step_sync, rcbf_safe_step (the hot
// path bench.py measures; kernel in rcbf_safe_step.hpp), rcbf_safe_step_seq,
// rcbf_safe_rollout, host buffers, version/ABI queries.
#include <atomic>

#include "rcbf_safe_step.hpp"

using namespace rcbf;

namespace {

template <int MODE>
__global__ void __launch_bounds__(kBlock) k_env_reset(rcbf_params prm, int64_t B, const uint8_t* __restrict__ mask,
                                                      const double* __restrict__ noise, uint64_t seed, int64_t off,
                                                      double* __restrict__ x, double* __restrict__ aux,
                                                      int32_t* __restrict__ step, uint32_t* __restrict__ episode,
                                                      float* __restrict__ obs_out) {
    using D = Dims<MODE, 1>;
    int64_t i = env_index();
    if (i < 0 || i >= B) return;
    if (mask && !mask[i]) return;
    double xs[D::NS], a;
    int st;
    uint32_t ep = episode ? episode[i] + 1u : 0u;
    env_reset_one<MODE>(noise, i, seed, off, ep, xs, a, st);
    store_state<MODE>(x, B, i, xs);
    aux[i] = a;
    step[i] = st;
    if (episode) episode[i] = ep;
    if (obs_out) store_obs32<MODE>(obs_out, i, xs);
}

template <int MODE, typename A>
__device__ __forceinline__ void env_step_one(const rcbf_params& prm, int64_t B, int64_t i, double* __restrict__ x,
                                             double* __restrict__ aux, int32_t* __restrict__ step,
                                             uint32_t* __restrict__ episode, const A* __restrict__ action,
                                             double* __restrict__ obs64, float* __restrict__ obs32,
                                             double* __restrict__ reward, double* __restrict__ cost,
                                             uint8_t* __restrict__ done, uint8_t* __restrict__ goal_met,
                                             int auto_reset, uint64_t seed, int64_t off) {
    using D = Dims<MODE, 1>;
    double xs[D::NS];
    load_state<MODE>(x, B, i, xs);
    double a = aux[i];
    int st = step[i];
    bool dn, gm = false;
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        CarsStepOut o;
        cars_env_step<A>(prm, xs, a, st, action[i], o);
        reward[i] = o.reward_d;
        cost[i] = o.cost;
        dn = o.done;
    } else {
        A act[2] = {action[2 * i], action[2 * i + 1]};
        UniStepOut o;
        uni_env_step<A>(prm, xs, a, st, act, o);
        reward[i] = o.reward;
        cost[i] = o.cost;
        dn = o.done;
        gm = o.goal;
    }
    done[i] = dn;
    if (goal_met) goal_met[i] = gm;
    if (auto_reset && dn) {
        uint32_t ep = episode ? episode[i] + 1u : 0u;
        env_reset_one<MODE>(nullptr, i, seed, off, ep, xs, a, st);
        if (episode) episode[i] = ep;
    }
    store_state<MODE>(x, B, i, xs);
    aux[i] = a;
    step[i] = st;
    if (obs64) {
        double o[D::NO];
        env_obs<MODE>(xs, o);
#pragma unroll
        for (int k = 0; k < D::NO; ++k) obs64[i * D::NO + k] = o[k];
    }
    if (obs32) store_obs32<MODE>(obs32, i, xs);
}

template <int MODE, typename A>
__global__ void __launch_bounds__(kBlock) k_env_step(rcbf_params prm, int64_t B, double* __restrict__ x,
                                                     double* __restrict__ aux, int32_t* __restrict__ step,
                                                     uint32_t* __restrict__ episode, const A* __restrict__ action,
                                                     double* __restrict__ obs64, float* __restrict__ obs32,
                                                     double* __restrict__ reward, double* __restrict__ cost,
                                                     uint8_t* __restrict__ done, uint8_t* __restrict__ goal_met,
                                                     int auto_reset, uint64_t seed, int64_t off) {
    int64_t i = env_index();
    if (i < 0 || i >= B) return;
    env_step_one<MODE, A>(prm, B, i, x, aux, step, episode, action, obs64, obs32, reward, cost, done, goal_met,
                          auto_reset, seed, off);
}

// The same step for one workgroup's worth of envs (B <= kBlock) whose results
// go to host memory (rcbf_env_step_sync): once every lane's outputs are
// written, one lane makes them visible system-wide and then stores `seq` to
// the host completion word, which the calling thread polls -- the call
// returns when the results are there, without waiting for the kernel-end
// cache actions and the completion signal behind hipStreamSynchronize.
template <int MODE, typename A>
__global__ void __launch_bounds__(kBlock) k_env_step_host(rcbf_params prm, int64_t B, double* __restrict__ x,
                                                          double* __restrict__ aux, int32_t* __restrict__ step,
                                                          uint32_t* __restrict__ episode, const A* __restrict__ action,
                                                          double* __restrict__ obs64, double* __restrict__ reward,
                                                          double* __restrict__ cost, uint8_t* __restrict__ done,
                                                          uint8_t* __restrict__ goal_met, int auto_reset, uint64_t seed,
                                                          int64_t off, uint32_t* done_word, uint32_t seq) {
    const int64_t i = threadIdx.x;  // one workgroup
    if (i < B)
        env_step_one<MODE, A>(prm, B, i, x, aux, step, episode, action, obs64, nullptr, reward, cost, done, goal_met,
                              auto_reset, seed, off);
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();  // every lane's host writes land before the word
        __hip_atomic_store(done_word, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_safe_rollout(rcbf_params prm, int64_t B, int Ksteps,
                                                         double* __restrict__ x, double* __restrict__ aux,
                                                         int32_t* __restrict__ step, uint32_t* __restrict__ episode,
                                                         const float* __restrict__ u_rl, float* __restrict__ obs_out,
                                                         float* __restrict__ reward_sum, float* __restrict__ cost_sum,
                                                         int32_t* __restrict__ n_done, int32_t* fail_flag,
                                                         uint64_t seed, int64_t off) {
    using D = Dims<MODE, K>;
    int64_t i = env_index();
    if (i < 0 || i >= B) return;
    double xs[D::NS];
    load_state<MODE>(x, B, i, xs);
    double a = aux[i];
    int st = step[i];
    float m[D::NS], s[D::NS];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        m[k] = 0.0f;
        s[k] = prior_sigma<MODE>(k);
    }
    float rs = 0.0f, cs = 0.0f;
    int nd = 0, worst = RCBF_QP_OK;
    for (int t = 0; t < Ksteps; ++t) {
        float us[D::NU], uf[D::NU];
#pragma unroll
        for (int c = 0; c < D::NU; ++c) us[c] = u_rl[((int64_t)t * B + i) * D::NU + c];
        float rew, cst;
        bool dn, gm;
        int status;
        safe_step_one<RCBF_SOLVER_ACTIVE_SET, MODE, K>(prm, i, xs, a, st, episode, us, m, s, uf, rew, cst, dn, gm,
                                                       status, 1, seed, off);
        rs += rew;
        cs += cst;
        nd += dn ? 1 : 0;
        worst = status > worst ? status : worst;
    }
    store_state<MODE>(x, B, i, xs);
    aux[i] = a;
    step[i] = st;
    if (obs_out) store_obs32<MODE>(obs_out, i, xs);
    reward_sum[i] = rs;
    cost_sum[i] = cs;
    n_done[i] = nd;
    if (worst != RCBF_QP_OK && fail_flag) atomicOr(fail_flag, 1 << worst);
}

}  // namespace

extern "C" {

const char* rcbf_version(void) { return "rcbf_hip 0.2.0 (gfx950)"; }
int32_t rcbf_abi_version(void) { return RCBF_ABI_VERSION; }
int32_t rcbf_params_size(void) { return (int32_t)sizeof(rcbf_params); }

int rcbf_env_reset(const rcbf_params* prm, int64_t B, const uint8_t* mask, const double* noise, uint64_t seed,
                   int64_t env_offset, double* x, double* aux, int32_t* step, uint32_t* episode, float* obs_out,
                   hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !aux || !step) return RCBF_E_NULL;
    if ((obs_out && (((uintptr_t)obs_out) & 7)) || (((uintptr_t)x) & 15)) return RCBF_E_BAD_SHAPE;
    if (prm->mode == RCBF_MODE_SIMULATED_CARS)
        hipLaunchKernelGGL((k_env_reset<RCBF_MODE_SIMULATED_CARS>), dim3(grid_for_envs(B)), dim3(kBlock), 0, stream, *prm,
                           B, mask, noise, seed, env_offset, x, aux, step, episode, obs_out);
    else
        hipLaunchKernelGGL((k_env_reset<RCBF_MODE_UNICYCLE>), dim3(grid_for_envs(B)), dim3(kBlock), 0, stream, *prm, B,
                           mask, noise, seed, env_offset, x, aux, step, episode, obs_out);
    return launch_status();
}

int rcbf_env_step(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step, uint32_t* episode,
                  const void* action, int32_t action_f64, double* obs64_out, float* obs_out, double* reward,
                  double* cost, uint8_t* done, uint8_t* goal_met, int32_t auto_reset, uint64_t seed,
                  int64_t env_offset, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !aux || !step || !action || !reward || !cost || !done) return RCBF_E_NULL;
    if ((obs_out && (((uintptr_t)obs_out) & 7)) || (((uintptr_t)x) & 15)) return RCBF_E_BAD_SHAPE;
    dim3 g(grid_for_envs(B)), b(kBlock);
#define RCBF_ENV_L(MODE, A)                                                                                       \
    hipLaunchKernelGGL((k_env_step<MODE, A>), g, b, 0, stream, *prm, B, x, aux, step, episode, (const A*)action, \
                       obs64_out, obs_out, reward, cost, done, goal_met, auto_reset, seed, env_offset)
    if (prm->mode == RCBF_MODE_SIMULATED_CARS) {
        if (action_f64)
            RCBF_ENV_L(RCBF_MODE_SIMULATED_CARS, double);
        else
            RCBF_ENV_L(RCBF_MODE_SIMULATED_CARS, float);
    } else {
        if (action_f64)
            RCBF_ENV_L(RCBF_MODE_UNICYCLE, double);
        else
            RCBF_ENV_L(RCBF_MODE_UNICYCLE, float);
    }
#undef RCBF_ENV_L
    return launch_status();
}

int rcbf_env_step_sync(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step, uint32_t* episode,
                       const void* action_host, int32_t action_f64, double* packed_host, int32_t auto_reset,
                       uint64_t seed, int64_t env_offset, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!packed_host) return RCBF_E_NULL;
    const int64_t no = prm->mode == RCBF_MODE_SIMULATED_CARS ? Dims<RCBF_MODE_SIMULATED_CARS, 1>::NO
                                                              : Dims<RCBF_MODE_UNICYCLE, 1>::NO;
    double* obs64 = packed_host;
    double* reward = packed_host + B * no;
    double* cost = reward + B;
    uint8_t* done = reinterpret_cast<uint8_t*>(cost + B);
    uint8_t* goal = done + B;
    if (B > kBlock) {  // several workgroups: wait for the stream
        int rc = rcbf_env_step(prm, B, x, aux, step, episode, action_host, action_f64, obs64, nullptr, reward, cost,
                               done, goal, auto_reset, seed, env_offset, stream);
        if (rc) return rc;
        return (int)hipStreamSynchronize(stream);
    }
    if (!x || !aux || !step || !action_host) return RCBF_E_NULL;
    if (((uintptr_t)x) & 15) return RCBF_E_BAD_SHAPE;
    // completion word: 4 bytes at the next 8-byte boundary after goal_met
    const int64_t word_off = (B * (8 * (no + 2) + 2) + 7) & ~int64_t(7);
    volatile uint32_t* word = reinterpret_cast<volatile uint32_t*>(reinterpret_cast<char*>(packed_host) + word_off);
    static std::atomic<uint32_t> counter{0};
    uint32_t seq = counter.fetch_add(1, std::memory_order_relaxed) + 1;
    if (seq == 0 || seq == *word) seq = counter.fetch_add(1, std::memory_order_relaxed) + 1;
#define RCBF_ENV_H(MODE, A)                                                                                         \
    hipLaunchKernelGGL((k_env_step_host<MODE, A>), dim3(1), dim3(kBlock), 0, stream, *prm, B, x, aux, step, episode, \
                       (const A*)action_host, obs64, reward, cost, done, goal, auto_reset, seed, env_offset,          \
                       (uint32_t*)word, seq)
    if (prm->mode == RCBF_MODE_SIMULATED_CARS) {
        if (action_f64)
            RCBF_ENV_H(RCBF_MODE_SIMULATED_CARS, double);
        else
            RCBF_ENV_H(RCBF_MODE_SIMULATED_CARS, float);
    } else {
        if (action_f64)
            RCBF_ENV_H(RCBF_MODE_UNICYCLE, double);
        else
            RCBF_ENV_H(RCBF_MODE_UNICYCLE, float);
    }
#undef RCBF_ENV_H
    if (int rc = launch_status()) return rc;
    // poll the word; every 4096 polls ask the stream, so a kernel that fails
    // (and never writes the word) returns its error instead of spinning
    for (uint32_t n = 1;; ++n) {
        if (*word == seq) return 0;
        __builtin_ia32_pause();
        if ((n & 4095) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) return *word == seq ? 0 : (int)hipErrorUnknown;
            if (q != hipErrorNotReady) return (int)q;
        }
    }
}

int rcbf_host_alloc(int64_t bytes, void** ptr) {
    if (!ptr) return RCBF_E_NULL;
    *ptr = nullptr;
    if (bytes <= 0) return RCBF_E_BAD_SHAPE;
    return (int)hipHostMalloc(ptr, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent);
}

int rcbf_host_free(void* ptr) { return ptr ? (int)hipHostFree(ptr) : 0; }

}  // extern "C"

namespace {

// One fused-step launch of the instantiation <SOLVER, MODE, K> at the
// workgroup size block_for_envs(B) picks; SPAN: the span-stamped entry point.
template <int SOLVER, int MODE, int K, bool SPAN = false>
void launch_k_safe_step(int64_t B, double* x, double* aux, int32_t* step, const float* u_rl, uint32_t* episode,
                        const float* mu, const float* sigma, float* obs_out, float* u_out, float* reward,
                        float* cost, uint8_t* done, uint8_t* goal_met, int32_t* status_out, int32_t* fail_flag,
                        int32_t auto_reset, uint64_t seed, int64_t env_offset, const rcbf_params& prm, int cols,
                        unsigned long long* span, hipStream_t stream) {
    // the exact (default) solver gets the small workgroups; the others run 256-thread ones
    const int bs = SOLVER == RCBF_SOLVER_ACTIVE_SET ? block_for_envs(B) : 256;
#define RCBF_SS_L(BS_)                                                                                             \
    hipLaunchKernelGGL((k_safe_step<SOLVER, MODE, K, false, BS_, SPAN>), dim3(grid_for_envs(B, BS_)), dim3(BS_), 0, \
                       stream, B, x, aux, step, u_rl, episode, mu, sigma, obs_out, u_out, reward, cost, done,       \
                       goal_met, status_out, fail_flag, auto_reset, seed, env_offset, prm, cols, span)
    if constexpr (SOLVER != RCBF_SOLVER_ACTIVE_SET) {
        RCBF_SS_L(256);
    } else {
        if (bs == 256)
            RCBF_SS_L(256);
        else if (bs == 128)
            RCBF_SS_L(128);
        else
            RCBF_SS_L(64);
    }
#undef RCBF_SS_L
}

int safe_step_launch(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step, uint32_t* episode,
                     const float* u_rl, const float* mu, const float* sigma, float* obs_out, float* u_out,
                     float* reward, float* cost, uint8_t* done, uint8_t* goal_met, int32_t* status_out,
                     int32_t* fail_flag, int32_t auto_reset, uint64_t seed, int64_t env_offset, int cols,
                     unsigned long long* span, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !aux || !step || !u_rl || !obs_out || !u_out || !reward || !cost || !done) return RCBF_E_NULL;
    if ((((uintptr_t)obs_out) & 7) || (((uintptr_t)x) & 15)) return RCBF_E_BAD_SHAPE;  // 8/16-B accesses
    if (span) {  // the measurement entry point: the default (exact active-set) solver only
        if (((uintptr_t)span) & 15) return RCBF_E_BAD_SHAPE;
        if (prm->solver != RCBF_SOLVER_ACTIVE_SET) return RCBF_E_BAD_MODE;
        constexpr int SOLVER_ = RCBF_SOLVER_ACTIVE_SET;
        RCBF_DISPATCH_MODE(prm, (launch_k_safe_step<SOLVER_, MODE_, K_, true>(
                                    B, x, aux, step, u_rl, episode, mu, sigma, obs_out, u_out, reward, cost, done,
                                    goal_met, status_out, fail_flag, auto_reset, seed, env_offset, *prm, cols, span,
                                    stream)));
    } else {
        RCBF_DISPATCH(prm, (launch_k_safe_step<SOLVER_, MODE_, K_>(B, x, aux, step, u_rl, episode, mu, sigma, obs_out,
                                                                   u_out, reward, cost, done, goal_met, status_out,
                                                                   fail_flag, auto_reset, seed, env_offset, *prm, cols,
                                                                   nullptr, stream)));
    }
    return launch_status();
}

}  // namespace

extern "C" {

int rcbf_safe_step(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step, uint32_t* episode,
                   const float* u_rl, const float* mu, const float* sigma, float* obs_out, float* u_out,
                   float* reward, float* cost, uint8_t* done, uint8_t* goal_met, int32_t* status_out,
                   int32_t* fail_flag, int32_t auto_reset, uint64_t seed, int64_t env_offset, hipStream_t stream) {
    return safe_step_launch(prm, B, x, aux, step, episode, u_rl, mu, sigma, obs_out, u_out, reward, cost, done,
                            goal_met, status_out, fail_flag, auto_reset, seed, env_offset, 0, nullptr, stream);
}

int rcbf_safe_step_span(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step, uint32_t* episode,
                        const float* u_rl, const float* mu, const float* sigma, int32_t prior_cols, float* obs_out,
                        float* u_out, float* reward, float* cost, uint8_t* done, uint8_t* goal_met,
                        int32_t* status_out, int32_t* fail_flag, int32_t auto_reset, uint64_t seed,
                        int64_t env_offset, uint64_t* span_out, hipStream_t stream) {
    if (!span_out) return RCBF_E_NULL;
    if (prior_cols && prm && prm->mode == RCBF_MODE_SIMULATED_CARS && mu) return RCBF_E_BAD_SHAPE;
    return safe_step_launch(prm, B, x, aux, step, episode, u_rl, mu, sigma, obs_out, u_out, reward, cost, done,
                            goal_met, status_out, fail_flag, auto_reset, seed, env_offset, prior_cols ? 1 : 0,
                            reinterpret_cast<unsigned long long*>(span_out), stream);
}

int rcbf_safe_step_cols(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step, uint32_t* episode,
                        const float* u_rl, const float* mu_cols, const float* sigma_cols, float* obs_out,
                        float* u_out, float* reward, float* cost, uint8_t* done, uint8_t* goal_met,
                        int32_t* status_out, int32_t* fail_flag, int32_t auto_reset, uint64_t seed,
                        int64_t env_offset, hipStream_t stream) {
    if (prm && prm->mode == RCBF_MODE_SIMULATED_CARS && mu_cols) return RCBF_E_BAD_SHAPE;  // the cars rows read no mean
    return safe_step_launch(prm, B, x, aux, step, episode, u_rl, mu_cols, sigma_cols, obs_out, u_out, reward, cost,
                            done, goal_met, status_out, fail_flag, auto_reset, seed, env_offset, 1, nullptr, stream);
}

}  // extern "C"

namespace {

int safe_step_seq_launch(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux, int32_t* step,
                         uint32_t* episode, const float* const* u_rl_seq, int32_t n_u_rl, const float* mu,
                         const float* sigma, int cols, float* obs_out, float* u_out, float* reward, float* cost,
                         uint8_t* done, uint8_t* goal_met, int32_t* status_out, int32_t* fail_flag,
                         int32_t auto_reset, uint64_t seed, int64_t env_offset, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0 || K < 0 || n_u_rl < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0 || K == 0) return 0;
    if (!u_rl_seq || n_u_rl == 0) return RCBF_E_NULL;
    for (int32_t j = 0; j < n_u_rl; ++j)
        if (!u_rl_seq[j]) return RCBF_E_NULL;
    if (!x || !aux || !step || !obs_out || !u_out || !reward || !cost || !done) return RCBF_E_NULL;
    if ((((uintptr_t)obs_out) & 7) || (((uintptr_t)x) & 15)) return RCBF_E_BAD_SHAPE;
    if (cols && prm->mode == RCBF_MODE_SIMULATED_CARS && mu) return RCBF_E_BAD_SHAPE;  // the cars rows read no mean
    RCBF_DISPATCH(prm, {
        for (int32_t j = 0; j < K; ++j) {
            launch_k_safe_step<SOLVER_, MODE_, K_>(B, x, aux, step, u_rl_seq[j % n_u_rl], episode, mu, sigma, obs_out,
                                                   u_out, reward, cost, done, goal_met, status_out, fail_flag,
                                                   auto_reset, seed, env_offset, *prm, cols, nullptr, stream);
            if (int e = launch_status()) return e;
        }
    });
    return 0;
}

}  // namespace

extern "C" {

int rcbf_safe_step_seq(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux, int32_t* step,
                       uint32_t* episode, const float* const* u_rl_seq, int32_t n_u_rl, const float* mu,
                       const float* sigma, float* obs_out, float* u_out, float* reward, float* cost, uint8_t* done,
                       uint8_t* goal_met, int32_t* status_out, int32_t* fail_flag, int32_t auto_reset, uint64_t seed,
                       int64_t env_offset, hipStream_t stream) {
    return safe_step_seq_launch(prm, B, K, x, aux, step, episode, u_rl_seq, n_u_rl, mu, sigma, 0, obs_out, u_out,
                                reward, cost, done, goal_met, status_out, fail_flag, auto_reset, seed, env_offset,
                                stream);
}

int rcbf_safe_step_seq_cols(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux, int32_t* step,
                            uint32_t* episode, const float* const* u_rl_seq, int32_t n_u_rl, const float* mu_cols,
                            const float* sigma_cols, float* obs_out, float* u_out, float* reward, float* cost,
                            uint8_t* done, uint8_t* goal_met, int32_t* status_out, int32_t* fail_flag,
                            int32_t auto_reset, uint64_t seed, int64_t env_offset, hipStream_t stream) {
    return safe_step_seq_launch(prm, B, K, x, aux, step, episode, u_rl_seq, n_u_rl, mu_cols, sigma_cols, 1, obs_out,
                                u_out, reward, cost, done, goal_met, status_out, fail_flag, auto_reset, seed,
                                env_offset, stream);
}

int rcbf_safe_rollout(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux, int32_t* step,
                      uint32_t* episode, const float* u_rl, float* obs_out, float* reward_sum, float* cost_sum,
                      int32_t* n_done, int32_t* fail_flag, uint64_t seed, int64_t env_offset, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0 || K < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0 || K == 0) return 0;
    if (!x || !aux || !step || !u_rl || !reward_sum || !cost_sum || !n_done) return RCBF_E_NULL;
    if ((obs_out && (((uintptr_t)obs_out) & 7)) || (((uintptr_t)x) & 15)) return RCBF_E_BAD_SHAPE;
    RCBF_DISPATCH_MODE(prm, hipLaunchKernelGGL((k_safe_rollout<MODE_, K_>), dim3(grid_for_envs(B)), dim3(kBlock), 0,
                                               stream, *prm, B, K, x, aux, step, episode, u_rl, obs_out, reward_sum,
                                               cost_sum, n_done, fail_flag, seed, env_offset));
    return launch_status();
}

}  // extern "C"
