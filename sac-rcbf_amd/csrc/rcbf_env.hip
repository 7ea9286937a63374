// rcbf_env.hip -- device-resident environments and the fused safe step + C-ABI:
// rcbf_env_reset, rcbf_env_step, rcbf_safe_step (the hot path bench.py
// measures), rcbf_safe_rollout, version/ABI queries.
//
// Env state is component-PAIR-major in HBM (see rcbf_common.hpp): one env per
// lane, each lane moves 16 B per component pair, and a wavefront's load or
// store of one pair is one contiguous 1 KiB access (dwordx4).  The fused step reads x, t, step, u_RL and
// writes x', t', step', obs (AoS, the policy's (B, n_o) input), u, reward,
// cost, done; the episode counter is touched only on resets.
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

template <int MODE>
__device__ __forceinline__ void load_state(const double* x, int64_t B, int64_t i, double* xs) {
    constexpr int NS = Dims<MODE, 1>::NS;
#pragma unroll
    for (int p = 0; p < NS / 2; ++p) {
        double2 v = ld_in2(&x[2 * (p * B + i)]);
        xs[2 * p] = v.x;
        xs[2 * p + 1] = v.y;
    }
    if constexpr (NS % 2) xs[NS - 1] = ld_in(&x[(NS - 1) * B + i]);
}

template <int MODE>
__device__ __forceinline__ void store_state(double* x, int64_t B, int64_t i, const double* xs) {
    constexpr int NS = Dims<MODE, 1>::NS;
#pragma unroll
    for (int p = 0; p < NS / 2; ++p) st_out2d(&x[2 * (p * B + i)], xs[2 * p], xs[2 * p + 1]);
    if constexpr (NS % 2) st_out(&x[(NS - 1) * B + i], xs[NS - 1]);
}

template <int MODE>
__device__ __forceinline__ void store_obs32(float* obs, int64_t i, const double* xs,
                                            const double* obs_cache = nullptr) {
    constexpr int NO = Dims<MODE, 1>::NO;
    double o[NO];
    if constexpr (MODE == RCBF_MODE_UNICYCLE && (kAblate & 8) == 0) {
        if (obs_cache && obs_cache[3] != 0.0)
            uni_obs_cs(xs, obs_cache[0], obs_cache[1], obs_cache[2], o);
        else
            env_obs<MODE>(xs, o);
    } else {
        env_obs<MODE>(xs, o);
    }
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        float* ov = obs + i * NO;  // 40 B rows, 8 B aligned
#pragma unroll
        for (int k = 0; k < NO / 2; ++k) st_out2(ov + 2 * k, (float)o[2 * k], (float)o[2 * k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < NO; ++k) st_out(&obs[i * NO + k], (float)o[k]);
    }
}

// Observation store through LDS (RCBF_OBS_STAGE=1): a full wave's 64 obs rows
// are one contiguous (64*NO*4)-byte block; lanes write their rows into LDS,
// then store the block as 16-byte chunks, chunk c by lane c%64 -- every
// store instruction covers whole contiguous lines (cars: 3 dwordx4 instead of
// 5 strided dwordx2).  Partial or unaligned waves take the per-lane path.
#ifndef RCBF_OBS_STAGE
#define RCBF_OBS_STAGE 1
#endif
template <int MODE>
__device__ __forceinline__ void store_obs32_staged(float* obs, int64_t i, int64_t B, const double* xs,
                                                   const double* obs_cache, float* lds_wave) {
    constexpr int NO = Dims<MODE, 1>::NO;
    const int lane = threadIdx.x & 63;
    const int64_t base = i - lane;
    const bool full = (kEnvsPerWave == 64) && (base + 64 <= B) && ((reinterpret_cast<uintptr_t>(obs) & 15) == 0);
    if (!full) {
        store_obs32<MODE>(obs, i, xs, obs_cache);
        return;
    }
    double o[NO];
    if constexpr (MODE == RCBF_MODE_UNICYCLE && (kAblate & 8) == 0) {
        if (obs_cache && obs_cache[3] != 0.0)
            uni_obs_cs(xs, obs_cache[0], obs_cache[1], obs_cache[2], o);
        else
            env_obs<MODE>(xs, o);
    } else {
        env_obs<MODE>(xs, o);
    }
    if constexpr (NO % 2 == 0) {
#pragma unroll
        for (int k = 0; k < NO / 2; ++k)
            *reinterpret_cast<float2*>(&lds_wave[lane * NO + 2 * k]) = make_float2((float)o[2 * k], (float)o[2 * k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < NO; ++k) lds_wave[lane * NO + k] = (float)o[k];
    }
    __builtin_amdgcn_wave_barrier();
    constexpr int CH = NO * 16;  // 16-byte chunks in the wave's block
    const float4* src = reinterpret_cast<const float4*>(lds_wave);
    float* dst = obs + base * NO;
#pragma unroll
    for (int j = 0; j < (CH + 63) / 64; ++j) {
        const int c = j * 64 + lane;
        if (CH % 64 == 0 || c < CH) st_out4(dst + 4 * c, src[c]);
    }
}

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
__global__ void __launch_bounds__(kBlock) k_env_step(rcbf_params prm, int64_t B, double* __restrict__ x,
                                                     double* __restrict__ aux, int32_t* __restrict__ step,
                                                     uint32_t* __restrict__ episode, const A* __restrict__ action,
                                                     double* __restrict__ obs64, float* __restrict__ obs32,
                                                     double* __restrict__ reward, double* __restrict__ cost,
                                                     uint8_t* __restrict__ done, uint8_t* __restrict__ goal_met,
                                                     int auto_reset, uint64_t seed, int64_t off) {
    using D = Dims<MODE, 1>;
    int64_t i = env_index();
    if (i < 0 || i >= B) return;
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

// Performance study: RCBF_WAVES_PER_EU=n tells the register allocator and the
// scheduler that n waves per SIMD suffice (the fused step runs one wave per
// SIMD at B = 65536), trading occupancy for instruction-level parallelism.
#ifdef RCBF_WAVES_PER_EU
#define RCBF_STEP_ATTR __attribute__((amdgpu_waves_per_eu(RCBF_WAVES_PER_EU, RCBF_WAVES_PER_EU)))
#else
#define RCBF_STEP_ATTR
#endif

template <int SOLVER, int MODE, int K>
__global__ void __launch_bounds__(kBlock) RCBF_STEP_ATTR k_safe_step(rcbf_params prm, int64_t B, double* __restrict__ x,
                                                      double* __restrict__ aux, int32_t* __restrict__ step,
                                                      uint32_t* __restrict__ episode, const float* __restrict__ u_rl,
                                                      const float* __restrict__ mu, const float* __restrict__ sigma,
                                                      float* __restrict__ obs_out, float* __restrict__ u_out,
                                                      float* __restrict__ reward, float* __restrict__ cost,
                                                      uint8_t* __restrict__ done, uint8_t* __restrict__ goal_met,
                                                      int32_t* __restrict__ status_out, int32_t* fail_flag,
                                                      int auto_reset, uint64_t seed, int64_t off) {
    using D = Dims<MODE, K>;
    int64_t i = env_index();
    if (i < 0 || i >= B) return;
#if RCBF_STAMPS
    unsigned long long* stamps = reinterpret_cast<unsigned long long*>(status_out);
    status_out = nullptr;
#else
    unsigned long long* stamps = nullptr;
#endif
    RCBF_STAMP(stamps, 0, false);
#ifdef RCBF_STAGGER  // performance study: odd workgroups start their loads later
    if (blockIdx.x & 1) __builtin_amdgcn_s_sleep(RCBF_STAGGER);
#endif
    double xs[D::NS];
    load_state<MODE>(x, B, i, xs);
    double a = ld_in(&aux[i]);
    int st = ld_in(&step[i]);
    float us[D::NU], m[D::NS], s[D::NS], uf[D::NU];
#pragma unroll
    for (int c = 0; c < D::NU; ++c) us[c] = ld_in(&u_rl[i * D::NU + c]);
    const bool ep_pre = episode && reset_foreseeable<MODE>(st, a);
    uint32_t ep0 = 0;
    if (ep_pre) ep0 = episode[i];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        m[k] = mu ? mu[i * D::NS + k] : 0.0f;
        s[k] = sigma ? sigma[i * D::NS + k] : prior_sigma<MODE>(k);
    }
    float rew, cst;
    bool dn, gm;
    int status;
    RCBF_STAMP(stamps, 1, true);
    double oc[4] = {0.0, 0.0, 0.0, 0.0};
    safe_step_one<SOLVER, MODE, K>(prm, i, xs, a, st, episode, us, m, s, uf, rew, cst, dn, gm, status, auto_reset,
                                   seed, off, stamps, oc, RCBF_EARLY_STORE ? u_out : nullptr, ep_pre, ep0);
    store_state<MODE>(x, B, i, xs);
    st_out(&aux[i], a);
    st_out(&step[i], st);
#if RCBF_OBS_STAGE
    __shared__ float obs_stage[kBlock / 64][64 * D::NO];
    store_obs32_staged<MODE>(obs_out, i, B, xs, oc, obs_stage[threadIdx.x >> 6]);
#else
    store_obs32<MODE>(obs_out, i, xs, oc);
#endif
#if !RCBF_EARLY_STORE
#pragma unroll
    for (int c = 0; c < D::NU; ++c) st_out(&u_out[i * D::NU + c], uf[c]);
#endif
    st_out(&reward[i], rew);
    st_out(&cost[i], cst);
    st_out(&done[i], (uint8_t)dn);
    if (goal_met) st_out(&goal_met[i], (uint8_t)gm);
    RCBF_STAMP(stamps, 6, false);
    report(status, status_out, i, fail_flag);
    RCBF_STAMP(stamps, 7, true);
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
    int rc = rcbf_env_step(prm, B, x, aux, step, episode, action_host, action_f64, obs64, nullptr, reward, cost, done,
                           goal, auto_reset, seed, env_offset, stream);
    if (rc) return rc;
    return (int)hipStreamSynchronize(stream);
}

int rcbf_host_alloc(int64_t bytes, void** ptr) {
    if (!ptr) return RCBF_E_NULL;
    *ptr = nullptr;
    if (bytes <= 0) return RCBF_E_BAD_SHAPE;
    return (int)hipHostMalloc(ptr, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent);
}

int rcbf_host_free(void* ptr) { return ptr ? (int)hipHostFree(ptr) : 0; }

int rcbf_safe_step(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step, uint32_t* episode,
                   const float* u_rl, const float* mu, const float* sigma, float* obs_out, float* u_out,
                   float* reward, float* cost, uint8_t* done, uint8_t* goal_met, int32_t* status_out,
                   int32_t* fail_flag, int32_t auto_reset, uint64_t seed, int64_t env_offset, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !aux || !step || !u_rl || !obs_out || !u_out || !reward || !cost || !done) return RCBF_E_NULL;
    if ((((uintptr_t)obs_out) & 7) || (((uintptr_t)x) & 15)) return RCBF_E_BAD_SHAPE;  // 8/16-B accesses
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_safe_step<SOLVER_, MODE_, K_>), dim3(grid_for_envs(B)), dim3(kBlock), 0,
                                          stream, *prm, B, x, aux, step, episode, u_rl, mu, sigma, obs_out, u_out,
                                          reward, cost, done, goal_met, status_out, fail_flag, auto_reset, seed,
                                          env_offset));
    return launch_status();
}

int rcbf_safe_step_seq(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux, int32_t* step,
                       uint32_t* episode, const float* const* u_rl_seq, int32_t n_u_rl, const float* mu,
                       const float* sigma, float* obs_out, float* u_out, float* reward, float* cost, uint8_t* done,
                       uint8_t* goal_met, int32_t* status_out, int32_t* fail_flag, int32_t auto_reset, uint64_t seed,
                       int64_t env_offset, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0 || K < 0 || n_u_rl < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0 || K == 0) return 0;
    if (!u_rl_seq || n_u_rl == 0) return RCBF_E_NULL;
    for (int32_t j = 0; j < n_u_rl; ++j)
        if (!u_rl_seq[j]) return RCBF_E_NULL;
    if (!x || !aux || !step || !obs_out || !u_out || !reward || !cost || !done) return RCBF_E_NULL;
    if ((((uintptr_t)obs_out) & 7) || (((uintptr_t)x) & 15)) return RCBF_E_BAD_SHAPE;
    RCBF_DISPATCH(prm, {
        for (int32_t j = 0; j < K; ++j) {
            hipLaunchKernelGGL((k_safe_step<SOLVER_, MODE_, K_>), dim3(grid_for_envs(B)), dim3(kBlock), 0, stream,
                               *prm, B, x, aux, step, episode, u_rl_seq[j % n_u_rl], mu, sigma, obs_out, u_out,
                               reward, cost, done, goal_met, status_out, fail_flag, auto_reset, seed, env_offset);
            if (int e = launch_status()) return e;
        }
    });
    return 0;
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
