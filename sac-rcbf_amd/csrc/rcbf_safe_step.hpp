// rcbf_safe_step.hpp -- the fused safe step kernel (the hot path bench.py
// measures) and the env-state / observation memory helpers it shares with
// the env kernels.  Included by rcbf_env.hip (the product instantiation) and
// by csrc/study/rcbf_stamps.hip (the phase-timing study build).
//
// Env state is component-PAIR-major in HBM (see rcbf_common.hpp): one env per
// lane, each lane moves 16 B per component pair, and a wavefront's load or
// store of one pair is one contiguous 1 KiB access (dwordx4).  The fused step
// reads x, t, step, u_RL and writes x', t', step', obs (AoS, the policy's
// (B, n_o) input), u, reward, cost, done; the episode counter is touched only
// on resets.
#pragma once

#include "rcbf_common.hpp"

// study override: prefetch this many argument lines in every mode
#ifndef RCBF_KARG_PREFETCH
#define RCBF_KARG_PREFETCH 0
#endif
// 1: the cars step stores the state pairs that do not depend on the safe
// action before the layer's chain runs (k_safe_step; 3.86 -> 3.67 us per
// step, profiles/r03/early_store_confirm_r03k.txt); 0: after it
#ifndef RCBF_EARLY_STORE
#define RCBF_EARLY_STORE 1
#endif

namespace rcbf {

// Touch each 64-B line of the first NL lines of the kernel argument block
// once, right after the state loads are issued, so the scalar loads of the
// parameters the compiler sinks into the body hit the scalar cache instead
// of each waiting for a miss on the critical path.  The global loads stay in
// flight across the one wait here.
template <int NL>
__device__ __forceinline__ void prefetch_kernargs() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t* ka = (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
    uint32_t acc = 0;
#pragma unroll
    for (int l = 0; l < NL; ++l) acc ^= ka[16 * l];
    asm volatile("" ::"s"(acc));
    __builtin_amdgcn_sched_barrier(0);
#endif
}

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

template <int MODE, bool WT = false>
__device__ __forceinline__ void store_obs32(float* obs, int64_t i, const double* xs,
                                            const double* obs_cache = nullptr) {
    constexpr int NO = Dims<MODE, 1>::NO;
    double o[NO];
    if constexpr (MODE == RCBF_MODE_UNICYCLE) {
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
        for (int k = 0; k < NO / 2; ++k) {
            if constexpr (WT) {
                const float pr[2] = {(float)o[2 * k], (float)o[2 * k + 1]};
                uint64_t w;
                __builtin_memcpy(&w, pr, 8);
                st_wt(reinterpret_cast<uint64_t*>(ov + 2 * k), w);
            } else {
                st_out2(ov + 2 * k, (float)o[2 * k], (float)o[2 * k + 1]);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NO; ++k) st_any<WT>(&obs[i * NO + k], (float)o[k]);
    }
}

// The wave's staged observation block (64 rows in LDS) to HBM as 16-byte
// chunks, chunk c by lane c % 64.  Every chunk is read from LDS first, then
// stored: the write-through store is an asm with a memory clobber, which
// would otherwise hold each following LDS read (and its wait) behind the
// previous store.
template <int MODE, bool WT = false>
__device__ __forceinline__ void store_obs_chunks(float* obs, int64_t base, const float* lds_wave) {
    constexpr int NO = Dims<MODE, 1>::NO;
    const int lane = threadIdx.x & 63;
    __builtin_amdgcn_wave_barrier();
    constexpr int CH = NO * 16;  // 16-byte chunks in the wave's block
    const float4* src = reinterpret_cast<const float4*>(lds_wave);
    float* dst = obs + base * NO;
    constexpr int NJ = (CH + 63) / 64;
    float4 chunk[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = j * 64 + lane;
        if (CH % 64 == 0 || c < CH) chunk[j] = src[c];
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = j * 64 + lane;
        if (CH % 64 == 0 || c < CH) st_out4<WT || MODE == RCBF_MODE_SIMULATED_CARS>(dst + 4 * c, chunk[j]);
    }
}

// Observation store through LDS: a full wave's 64 obs rows are one
// contiguous (64*NO*4)-byte block; lanes write their rows into LDS, then
// store the block as 16-byte chunks, chunk c by lane c%64 -- every store
// instruction covers whole contiguous lines (cars: 3 dwordx4 instead of 5
// strided dwordx2).  Partial or unaligned waves take the per-lane path.
template <int MODE, bool WT = false>
__device__ __forceinline__ void store_obs32_staged(float* obs, int64_t i, int64_t B, const double* xs,
                                                   const double* obs_cache, float* lds_wave) {
    constexpr int NO = Dims<MODE, 1>::NO;
    const int lane = threadIdx.x & 63;
    const int64_t base = i - lane;
#ifdef RCBF_STUDY_EPW  // study: a 64-thread workgroup's wave holds fewer than 64 envs (per-lane stores)
    const bool full = blockDim.x != 64 && (base + 64 <= B) && ((reinterpret_cast<uintptr_t>(obs) & 15) == 0);
#else
    const bool full = (base + 64 <= B) && ((reinterpret_cast<uintptr_t>(obs) & 15) == 0);
#endif
    if (!full) {
        store_obs32<MODE, WT>(obs, i, xs, obs_cache);
        return;
    }
    double o[NO];
    if constexpr (MODE == RCBF_MODE_UNICYCLE) {
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
    store_obs_chunks<MODE, WT>(obs, base, lds_wave);
}

// The fused safe step (rcbf_safe_step): one env per lane.  ST = true only in
// the study build (csrc/study/rcbf_stamps.hip), which records phase
// timestamps into `stamps`; the product instantiation ignores it.
// BS: workgroup size (block_for_envs).  SPAN = true (rcbf_safe_step_span, a
// measurement entry point of the product library): lane 0 of every wave
// writes the chip clock (s_memrealtime, 100 MHz) at its start and after its
// own stores have completed to stamp_buf[4 w], [4 w + 1], and the shader
// clock (s_memtime) at the same two points to stamp_buf[4 w + 2], [4 w + 3]
// (the clock the wave ran at is delta(s_memtime) / delta(s_memrealtime) x
// 100 MHz); every other instruction is the product's.
// Argument order: B and the pointers of the first loads lead (one 64-B line
// of the argument block, which the launch can preload into SGPRs), the
// parameter block comes last.
template <int SOLVER, int MODE, int K, bool ST = false, int BS = kBlock, bool SPAN = false>
__global__ void __launch_bounds__(BS) k_safe_step(int64_t B, double* __restrict__ x, double* __restrict__ aux,
                                                      int32_t* __restrict__ step, const float* __restrict__ u_rl,
                                                      uint32_t* __restrict__ episode, const float* __restrict__ mu,
                                                      const float* __restrict__ sigma, float* __restrict__ obs_out,
                                                      float* __restrict__ u_out, float* __restrict__ reward,
                                                      float* __restrict__ cost, uint8_t* __restrict__ done,
                                                      uint8_t* __restrict__ goal_met,
                                                      int32_t* __restrict__ status_out, int32_t* fail_flag,
                                                      int auto_reset, uint64_t seed, int64_t off, rcbf_params prm,
                                                      int prior_cols = 0, unsigned long long* stamp_buf = nullptr) {
    using D = Dims<MODE, K>;
    // RCBF_WT_OUT: every output write-through, the wave's stores drained before
    // it ends (rcbf_common.hpp, WtStage); the study stamps build keeps the nt form
    constexpr bool WT = RCBF_WT_OUT != 0 && !ST;
    int64_t i = env_index<BS>();
    if (i >= B) return;
    const int lane = threadIdx.x & 63;
    const int64_t wbase = i - lane;
    const bool wfull = wbase + 64 <= B;  // wave-uniform: every lane of this wave is live
    constexpr int kWtBytes = WT ? 16 * 160 : 16;  // per wave: the largest WtStage below (unicycle, 152 chunks)
    __shared__ __attribute__((aligned(16))) char wt_lds_all[BS / 64][kWtBytes];
    char* wt_lds = wt_lds_all[threadIdx.x >> 6];
    (void)wt_lds;
    (void)wfull;
    unsigned long long span_t0 = 0, span_c0 = 0;
    if constexpr (SPAN) {
        span_t0 = __builtin_amdgcn_s_memrealtime();
        span_c0 = __builtin_amdgcn_s_memtime();
    }
    Stamps<ST> stamps;
    stamps.buf = stamp_buf;
    stamps.mark(0, false);
    double xs[D::NS];
    load_state<MODE>(x, B, i, xs);
    double a = ld_in(&aux[i]);
    int st = ld_in(&step[i]);
    float us[D::NU], m[D::NS], s[D::NS], uf[D::NU];
#pragma unroll
    for (int c = 0; c < D::NU; ++c) us[c] = ld_in(&u_rl[i * D::NU + c]);
#if RCBF_KARG_PREFETCH
    prefetch_kernargs<RCBF_KARG_PREFETCH>();
#else
    // cars: 3.87 -> 3.81 us per step; the unicycle step is slower with it
    // (4.38 -> 4.50 us at k = 5; profiles/r03/kernarg_preload_ab_r03d.txt)
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) prefetch_kernargs<7>();
#endif
    const bool ep_pre = episode && reset_foreseeable<MODE>(st, a);
    uint32_t ep0 = 0;
    if (ep_pre) ep0 = episode[i];
    if (prior_cols) {
        // column layout (rcbf_safe_step_cols): only what the rows read, one
        // contiguous (B,) f32 column each -- cars sigma (3, B) = sigma[:, 5],
        // [:, 7], [:, 9] (the cars rows ignore mu, diff_cbf_qp.py:298-299);
        // unicycle mu and sigma (3, B)
#pragma unroll
        for (int k = 0; k < D::NS; ++k) {
            m[k] = 0.0f;
            s[k] = prior_sigma<MODE>(k);
        }
        if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
            if (sigma) {
                s[5] = ld_in(&sigma[i]);
                s[7] = ld_in(&sigma[B + i]);
                s[9] = ld_in(&sigma[2 * B + i]);
            }
        } else {
#pragma unroll
            for (int k = 0; k < D::NS; ++k) {
                if (mu) m[k] = ld_in(&mu[k * B + i]);
                if (sigma) s[k] = ld_in(&sigma[k * B + i]);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < D::NS; ++k) {
            m[k] = mu ? mu[i * D::NS + k] : 0.0f;
            s[k] = sigma ? sigma[i * D::NS + k] : prior_sigma<MODE>(k);
        }
    }
    float rew, cst;
    bool dn, gm;
    int status;
    stamps.mark(1, true);
    double oc[4] = {0.0, 0.0, 0.0, 0.0};
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS && RCBF_EARLY_STORE && !ST) {
        // The same step in an order that lets 76 of the 145 written bytes
        // leave while the layer's chain is still running: the env's
        // pre-step part (everything but car 3's velocity, t, step, done,
        // cost) and the auto-reset do not depend on the safe action, so
        // they, and the stores of state pairs 0, 1, 2, 4, t and step, come
        // first; the layer's chain (state32 -> rows -> QP -> clamp) then
        // finishes car 3's velocity (pair 3) and the observation.
        float s32[D::NS];
        state_from_env<MODE>(xs, s32);  // the layer reads the pre-step state
        // the exact solver on the raw rows: the rows are built here, ahead of
        // the env's pre-step part, whose arithmetic can then fill their latency
        // (3.69 -> 3.65 us per step, profiles/r03/rows_first_ab_r03q.txt)
        constexpr bool kRowsFirst = SOLVER == RCBF_SOLVER_ACTIVE_SET && RCBF_FUSED_RAW_ROWS != 0;
        LayerState<MODE, K> L;
        if constexpr (kRowsFirst) diff_rows<MODE, K>(prm, s32, us, m, s, L.G, L.h, nullptr);
        CarsStepOut o;
        const double acc3 = cars_env_pre(prm, xs, a, st, o);
        dn = o.done;
        cst = (float)o.cost;
        gm = false;
        const bool rs = auto_reset && dn;
        if (rs) {
            const uint32_t ep = episode ? (ep_pre ? ep0 : episode[i]) + 1u : 0u;
            if (episode) {
                if constexpr (WT)
                    st_wt(&episode[i], ep);
                else
                    episode[i] = ep;
            }
            env_reset_one<MODE>(nullptr, i, seed, off, ep, xs, a, st);
        }
#pragma unroll
        for (int p = 0; p < D::NS / 2; ++p)
            if (p != 3) st_any2d<WT>(&x[2 * (p * B + i)], xs[2 * p], xs[2 * p + 1]);
        if constexpr (WT) {
            using E = WtStage<8, 4>;  // aux, step
            char* const dst[2] = {reinterpret_cast<char*>(aux + wbase), reinterpret_cast<char*>(step + wbase)};
            const uint64_t val[2] = {wt_bits(a), wt_bits(st)};
            E::store(wt_lds, lane, wfull, dst, val);
        } else {
            st_out(&aux[i], a);
            st_out(&step[i], st);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the early stores ahead of the layer's chain
        if constexpr (kRowsFirst) {
            layer_solve_raw<MODE, K>(prm, us, uf, L);  // the same solve as layer_forward<..., RAW>
        } else {
            layer_forward<SOLVER, MODE, K, false, false, RCBF_FUSED_RAW_ROWS != 0>(prm, s32, us, m, s, uf, L);
        }
        status = L.qp.status;
        const double v3_reset = xs[7];
        cars_env_post<float>(xs, acc3, uf[0], o);  // car 3's velocity and the reward
        xs[7] = rs ? v3_reset : xs[7];
        rew = o.reward;
        st_any2d<WT>(&x[2 * (3 * B + i)], xs[6], xs[7]);
    } else {
        safe_step_one<SOLVER, MODE, K, ST, WT>(prm, i, xs, a, st, episode, us, m, s, uf, rew, cst, dn, gm, status,
                                               auto_reset, seed, off, stamps, oc, ep_pre, ep0);
        if constexpr (WT) {
#pragma unroll
            for (int p = 0; p < D::NS / 2; ++p) st_wt2d(&x[2 * (p * B + i)], xs[2 * p], xs[2 * p + 1]);
            // the odd component (unicycle theta), aux and step leave with the outputs below
        } else {
            store_state<MODE>(x, B, i, xs);
            st_out(&aux[i], a);
            st_out(&step[i], st);
        }
    }
    __shared__ float obs_stage[BS / 64][64 * D::NO];
    store_obs32_staged<MODE, WT>(obs_out, i, B, xs, oc, obs_stage[threadIdx.x >> 6]);
    if constexpr (WT) {
        constexpr int NU4 = 4 * D::NU;
        float ufc[D::NU];
#pragma unroll
        for (int c = 0; c < D::NU; ++c) ufc[c] = uf[c];
        char* const u_d = reinterpret_cast<char*>(u_out + wbase * D::NU);
        char* const r_d = reinterpret_cast<char*>(reward + wbase);
        char* const c_d = reinterpret_cast<char*>(cost + wbase);
        char* const d_d = reinterpret_cast<char*>(done + wbase);
        uint64_t u_v = 0;
        __builtin_memcpy(&u_v, ufc, sizeof(ufc));
        const uint64_t r_v = wt_bits(rew), c_v = wt_bits(cst), d_v = (uint64_t)dn;
        if constexpr (MODE == RCBF_MODE_SIMULATED_CARS && RCBF_EARLY_STORE) {
            if (goal_met) {
                using E = WtStage<NU4, 4, 4, 1, 1>;
                char* const dst[5] = {u_d, r_d, c_d, d_d, reinterpret_cast<char*>(goal_met + wbase)};
                const uint64_t val[5] = {u_v, r_v, c_v, d_v, (uint64_t)gm};
                E::store(wt_lds, lane, wfull, dst, val);
            } else {
                using E = WtStage<NU4, 4, 4, 1>;
                char* const dst[4] = {u_d, r_d, c_d, d_d};
                const uint64_t val[4] = {u_v, r_v, c_v, d_v};
                E::store(wt_lds, lane, wfull, dst, val);
            }
        } else {
            static_assert(D::NS % 2 == 1, "the late write-through block carries the odd state component");
            char* const x_d = reinterpret_cast<char*>(x + (D::NS - 1) * B + wbase);
            char* const a_d = reinterpret_cast<char*>(aux + wbase);
            char* const s_d = reinterpret_cast<char*>(step + wbase);
            const uint64_t x_v = wt_bits(xs[D::NS - 1]), a_v = wt_bits(a), s_v = wt_bits(st);
            if (goal_met) {
                using E = WtStage<8, 8, 4, NU4, 4, 4, 1, 1>;
                static_assert(E::kBytes <= kWtBytes, "wt_lds");
                char* const dst[8] = {x_d, a_d, s_d, u_d, r_d, c_d, d_d, reinterpret_cast<char*>(goal_met + wbase)};
                const uint64_t val[8] = {x_v, a_v, s_v, u_v, r_v, c_v, d_v, (uint64_t)gm};
                E::store(wt_lds, lane, wfull, dst, val);
            } else {
                using E = WtStage<8, 8, 4, NU4, 4, 4, 1>;
                char* const dst[7] = {x_d, a_d, s_d, u_d, r_d, c_d, d_d};
                const uint64_t val[7] = {x_v, a_v, s_v, u_v, r_v, c_v, d_v};
                E::store(wt_lds, lane, wfull, dst, val);
            }
        }
    } else {
#pragma unroll
        for (int c = 0; c < D::NU; ++c) st_out(&u_out[i * D::NU + c], uf[c]);
        st_out(&reward[i], rew);
        st_out(&cost[i], cst);
        st_out(&done[i], (uint8_t)dn);
        if (goal_met) st_out(&goal_met[i], (uint8_t)gm);
    }
    stamps.mark(6, false);
    if constexpr (WT) {
        if (status_out) st_wt(&status_out[i], (int32_t)status);
        if (status != RCBF_QP_OK && fail_flag) atomicOr(fail_flag, 1 << status);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing this wave wrote is in flight when it ends
    } else {
        report(status, status_out, i, fail_flag);
    }
    stamps.mark(7, true);
    if constexpr (SPAN) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have landed
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long c1 = __builtin_amdgcn_s_memtime();
        if ((threadIdx.x & 63) == 0) {
            const int64_t w = ((int64_t)blockIdx.x * BS + threadIdx.x) >> 6;
            typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<u2*>(stamp_buf + 4 * w) = u2{span_t0, t1};
            *reinterpret_cast<u2*>(stamp_buf + 4 * w + 2) = u2{span_c0, c1};
        }
    }
}

}  // namespace rcbf
