// rcbf_common.hpp -- pieces shared by the three kernel translation units
// (rcbf_layer.hip, rcbf_qp.hip, rcbf_env.hip): mode traits, the fused
// CBFQPLayer forward for one env, env helpers, launch/dispatch helpers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <type_traits>

#include "rcbf_device.hpp"

// The fused step solves the raw CBF rows (layer_forward's RAW); 0 restores
// the normalised rows (the A/B build of the study).
#ifndef RCBF_FUSED_RAW_ROWS
#define RCBF_FUSED_RAW_ROWS 1
#endif

namespace rcbf {

constexpr int kBlock = 256;

inline unsigned grid_for(int64_t B) { return (unsigned)((B + kBlock - 1) / kBlock); }
inline unsigned grid_for_envs(int64_t B) { return grid_for(B); }

// env index of this lane in the env kernels: one env per lane
#ifndef RCBF_STUDY_EPW
template <int BS = kBlock>
__device__ __forceinline__ int64_t env_index() { return (int64_t)blockIdx.x * BS + threadIdx.x; }
#else
// study build (scripts/epw_study.sh): the one-wave (64-thread) workgroups of small batches carry only
// RCBF_STUDY_EPW envs, on lanes 0 .. EPW - 1 (the rest exit: their index is past any B), so a batch
// reaches 64 / EPW times as many CUs
template <int BS = kBlock>
__device__ __forceinline__ int64_t env_index() {
    if constexpr (BS == 64)
        return threadIdx.x < RCBF_STUDY_EPW ? (int64_t)blockIdx.x * RCBF_STUDY_EPW + threadIdx.x : INT64_MAX;
    return (int64_t)blockIdx.x * BS + threadIdx.x;
}
#endif

// Workgroup size of the fused step for a batch of B envs.  The step is a
// per-CU memory-request-bound chain at one wave per SIMD (half
// the batch on half the CUs takes the same time), so a batch that would leave
// CUs without a 256-thread workgroup (B < 256 CUs x 256) is cut into smaller
// workgroups that reach more CUs: 128 threads for B >= 32 768 (256-511
// workgroups), 64 below (one wave per workgroup).
// CUs of the current device (256 on an MI355X), queried once per device
// ordinal and cached: the thresholds follow the part (or partition mode) the
// launch actually runs on.
inline int64_t num_cus() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int cus = cache[dev].load(std::memory_order_relaxed);
    if (cus <= 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        cache[dev].store(cus, std::memory_order_relaxed);
    }
    return cus;
}
#ifndef RCBF_STUDY_BLOCK256  // study build: 256-thread workgroups at every batch (the r03 launch)
inline int block_for_envs(int64_t B) {
    const int64_t cus = num_cus();
    return B >= cus * 256 ? 256 : B >= cus * 128 ? 128 : 64;
}
#else
inline int block_for_envs(int64_t) { return 256; }
#endif
#ifndef RCBF_STUDY_EPW
inline unsigned grid_for_envs(int64_t B, int bs) { return (unsigned)((B + bs - 1) / bs); }
#else
inline unsigned grid_for_envs(int64_t B, int bs) {
    const int e = bs == 64 ? RCBF_STUDY_EPW : bs;
    return (unsigned)((B + e - 1) / e);
}
#endif

// Memory policy of the env kernels: every once-read input is an `nt` load and
// every output an `nt` store (with the whole-line stores below the fastest of
// the flavours measured: plain, write-through sc1, nt; profiles/r01).
template <typename T>
__device__ __forceinline__ void st_out(T* p, T v) {
    __builtin_nontemporal_store(v, p);
}

// 16-byte store (staged observation chunks).  WT: write-through (`sc1`), the
// line leaves the XCD's L2 as it is written instead of waiting, dirty, for the
// kernel-end write-back.  The cars step takes it (4.40 -> 4.18 us per step,
// rocprof-traced 5.26 -> 5.03 us; profiles/r02/obs_store_flavours_r02m.txt);
// the unicycle step is slower with it (5.08 -> 5.41 us) and keeps `nt`.
template <bool WT = false>
__device__ __forceinline__ void st_out4(float* p, float4 v) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 w = {v.x, v.y, v.z, v.w};
    if constexpr (WT) {
        // the s_nop covers the store-data hazard the compiler cannot see inside the asm
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
    } else {
        __builtin_nontemporal_store(w, reinterpret_cast<f4*>(p));
    }
}

// 16-byte f64 pair store (env state pairs)
__device__ __forceinline__ void st_out2d(double* p, double a, double b) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 w = {a, b};
    __builtin_nontemporal_store(w, reinterpret_cast<d2*>(p));
}

template <typename T>
__device__ __forceinline__ T ld_in(const T* p) {
    return __builtin_nontemporal_load(p);
}

__device__ __forceinline__ double2 ld_in2(const double* p) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2*>(p));
    return make_double2(v.x, v.y);
}

// 8-byte pair store (obs rows): one dwordx2 store
__device__ __forceinline__ void st_out2(float* p, float a, float b) {
    union {
        float f[2];
        uint64_t u;
    } w;
    w.f[0] = a;
    w.f[1] = b;
    st_out<uint64_t>(reinterpret_cast<uint64_t*>(p), w.u);
}

// ---------------------------------------------------------------------------
// STUDY BUILD (-DRCBF_WT_OUT=1, scripts/exp_wt_nofence.py; the product is
// RCBF_WT_OUT=0 and its machine code is unchanged by this block).  Measured
// r06l (profiles/r06/wt_nofence_r06l.txt): the write-through stores cost the
// cars step 1.35 us of in-kernel span (2.56 -> 3.91) to save 0.4-0.7 us of
// boundary, so 3.88 -> 4.56-4.63 us per step; not adopted.
// Write-through outputs of the fused step (RCBF_WT_OUT).  Every byte the step
// writes leaves the XCD's L2 as it is stored (`sc1`), and each wave waits for
// its stores before it ends, so when the dispatch completes nothing it wrote is
// dirty in any L2: the next step (an AQL packet with an agent-scope acquire and
// NO release, csrc/rcbf_aql.hip) reads it from the coherent side on whichever
// XCD it runs, and two XCDs never hold dirty copies of one output line.  The
// per-step L2 write-back of the kernel-end release is what it removes
// (DESIGN §3.5).  Narrow `sc1` stores are one fabric write per lane, so the
// per-env scalars of a full wave are staged in LDS and leave as 16-B chunks
// (WtStage).
// ---------------------------------------------------------------------------
#ifndef RCBF_WT_OUT
#define RCBF_WT_OUT 0
#endif

// 16-byte write-through store of two doubles (a state pair)
__device__ __forceinline__ void st_wt2d(double* p, double a, double b) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 w = {a, b};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
}

// one lane's write-through store of a 1/4/8-byte value (partial waves, rare stores)
template <typename T>
__device__ __forceinline__ void st_wt(T* p, T v) {
    static_assert(sizeof(T) == 1 || sizeof(T) == 4 || sizeof(T) == 8, "st_wt: 1, 4 or 8 bytes");
    using U = typename std::conditional<sizeof(T) == 1, uint8_t,
                                        typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type>::type;
    U u;
    __builtin_memcpy(&u, &v, sizeof(T));
    __hip_atomic_store(reinterpret_cast<U*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the store flavour of one output: write-through under WT, `nt` otherwise
template <bool WT, typename T>
__device__ __forceinline__ void st_any(T* p, T v) {
    if constexpr (WT)
        st_wt(p, v);
    else
        st_out(p, v);
}
template <bool WT>
__device__ __forceinline__ void st_any2d(double* p, double a, double b) {
    if constexpr (WT)
        st_wt2d(p, a, b);
    else
        st_out2d(p, a, b);
}

// Staged write-through of a full wave's per-env scalars.  Segment s holds one
// SZ_s-byte value per lane; the wave's 64 values of a segment are one
// contiguous (64 SZ_s)-byte block at dst_s (= array + first env of the wave x
// SZ_s), i.e. 4 SZ_s chunks of 16 B.  The LDS block mirrors the chunk order
// (segment s at byte 16 pre_s), so chunk c is read from lds + 16 c and goes to
// dst_s + 16 (c - pre_s), the chunks of every segment dealt over the lanes
// together: a handful of dwordx4 `sc1` stores per wave instead of one narrow
// fabric write per lane and output.
template <int... SZ>
struct WtStage {
    static constexpr int kN = sizeof...(SZ);
    static constexpr int kSz[kN] = {SZ...};
    static constexpr int pre(int s) {
        int p = 0;
        for (int j = 0; j < s; ++j) p += 4 * kSz[j];
        return p;
    }
    static constexpr int kChunks = pre(kN);
    static constexpr int kBytes = 16 * kChunks;
    // lane deposits its value of segment S
    template <int S, typename T>
    static __device__ __forceinline__ void put(char* lds, int lane, T v) {
        static_assert(sizeof(T) == kSz[S], "WtStage::put: value size");
        *reinterpret_cast<T*>(lds + 16 * pre(S) + lane * (int)sizeof(T)) = v;
    }
    // the wave's chunks to HBM (all lanes of the wave call it)
    static __device__ __forceinline__ void flush(const char* lds, int lane, char* const (&dst)[kN]) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_wave_barrier();
        constexpr int NJ = (kChunks + 63) / 64;
        f4 v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int c = j * 64 + lane;
            if (kChunks % 64 == 0 || c < kChunks) v[j] = reinterpret_cast<const f4*>(lds)[c];
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int c = j * 64 + lane;
            if (kChunks % 64 == 0 || c < kChunks) {
                char* d = nullptr;
#pragma unroll
                for (int s = 0; s < kN; ++s)
                    if (c >= pre(s) && c < pre(s + 1)) d = dst[s] + 16 * (c - pre(s));
                asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(d), "v"(v[j]) : "memory");
            }
        }
    }
    // true when every segment's block of this wave is 16-B aligned
    static __device__ __forceinline__ bool aligned(char* const (&dst)[kN]) {
        uintptr_t a = 0;
#pragma unroll
        for (int s = 0; s < kN; ++s) a |= reinterpret_cast<uintptr_t>(dst[s]);
        return (a & 15) == 0;
    }
    // The whole store: val[s] holds this lane's value of segment s in its low
    // SZ_s bytes; dst[s] = the segment's array + the wave's first env x SZ_s.
    // full: all 64 lanes of the wave are live (wave-uniform); otherwise, or
    // when a block is unaligned, every lane stores its own values write-through.
    static __device__ __forceinline__ void store(char* lds, int lane, bool full, char* const (&dst)[kN],
                                                 const uint64_t (&val)[kN]) {
        if (full && aligned(dst)) {
#pragma unroll
            for (int s = 0; s < kN; ++s) {
                char* q = lds + 16 * pre(s) + lane * kSz[s];
                if (kSz[s] == 8) *reinterpret_cast<uint64_t*>(q) = val[s];
                else if (kSz[s] == 4) *reinterpret_cast<uint32_t*>(q) = (uint32_t)val[s];
                else *reinterpret_cast<uint8_t*>(q) = (uint8_t)val[s];
            }
            flush(lds, lane, dst);
        } else {
#pragma unroll
            for (int s = 0; s < kN; ++s) {
                char* q = dst[s] + lane * kSz[s];
                if (kSz[s] == 8) st_wt(reinterpret_cast<uint64_t*>(q), val[s]);
                else if (kSz[s] == 4) st_wt(reinterpret_cast<uint32_t*>(q), (uint32_t)val[s]);
                else st_wt(reinterpret_cast<uint8_t*>(q), (uint8_t)val[s]);
            }
        }
    }
};

// the low bytes of a value as a WtStage::store operand
template <typename T>
__device__ __forceinline__ uint64_t wt_bits(T v) {
    static_assert(sizeof(T) <= 8 && !std::is_pointer<T>::value, "wt_bits: a scalar value");
    uint64_t u = 0;
    __builtin_memcpy(&u, &v, sizeof(T));
    return u;
}

// Phase timestamps of the fused step for the study build only
// (csrc/study/rcbf_stamps.hip, scripts/stamps.py): lane 0 of every wave
// records s_memtime at phase boundaries into buf as uint64 [wave][16], and
// s_memrealtime (one 100 MHz clock for the whole chip) at its start and end.  The
// product kernels use Stamps<false>, whose mark() compiles to nothing.
template <bool ON>
struct Stamps {
    unsigned long long* buf = nullptr;
    __device__ __forceinline__ void mark(int j, bool drain) const {
        if constexpr (ON) {
            if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long t;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            __builtin_amdgcn_sched_barrier(0);
            if ((threadIdx.x & 63) == 0 && buf) buf[((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 16 + j] = t;
            if (j == 0 || j == 7) {  // the chip-wide 100 MHz clock at wave start / end, slots 10 / 11
                const unsigned long long rt = __builtin_amdgcn_s_memrealtime();
                if ((threadIdx.x & 63) == 0 && buf)
                    buf[((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 16 + (j == 0 ? 10 : 11)] = rt;
            }
        }
    }
    __device__ __forceinline__ void count(int j, bool lane_flag) const {
        if constexpr (ON) {
            unsigned long long b = __ballot(lane_flag);
            if ((threadIdx.x & 63) == 0 && buf) buf[((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 16 + j] = __popcll(b);
        }
    }
};

// ---------------------------------------------------------------------------
// mode traits
// ---------------------------------------------------------------------------
template <int MODE, int K>
struct Dims;
template <int K>
struct Dims<RCBF_MODE_SIMULATED_CARS, K> {
    static constexpr int NS = 10, NU = 1, N = 2, M = 4, NO = 10;
};
template <int K>
struct Dims<RCBF_MODE_UNICYCLE, K> {
    static constexpr int NS = 3, NU = 2, N = 3, M = K + 4, NO = 7;
};

// prior disturbance (dynamics.py:24, 381-384): mean 0, sigma = MAX_STD cast to fp32
template <int MODE>
__device__ __forceinline__ float prior_sigma(int k) {
    if (MODE == RCBF_MODE_SIMULATED_CARS) return (k & 1) ? (float)0.2 : 0.0f;
    return (float)0.2;
}

// P of the diff layer, as the fp32 tensor qpth receives then casts to fp64
// (diff_cbf_qp.py:265,356,139)
template <int MODE>
__device__ __forceinline__ void diff_P(double* d) {
    if (MODE == RCBF_MODE_SIMULATED_CARS) {
        d[0] = (double)0.1f;
        d[1] = (double)10.0f;
    } else {
        d[0] = (double)1.0f;
        d[1] = (double)1e-2f;
        d[2] = (double)1e5f;
    }
}

// P of the Cascade layer (cbf_qp.py:146, 218), fp64
template <int MODE>
__device__ __forceinline__ void cascade_P(double* d) {
    if (MODE == RCBF_MODE_SIMULATED_CARS) {
        d[0] = 0.1;
        d[1] = 1e1;
    } else {
        d[0] = 1.e1;
        d[1] = 1.e-4;
        d[2] = 1e7;
    }
}

// cs_row [unicycle, nullable]: fp32 cos/sin of xs[2] already known (the fused step)
template <int MODE, int K>
__device__ __forceinline__ void diff_rows(const rcbf_params& prm, const float* xs, const float* u,
                                          const float* mu, const float* sig,
                                          float (*G)[Dims<MODE, K>::N], float* h, const float* cs_row = nullptr) {
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        cars_rows_diff(prm, xs, u[0], sig[5], sig[7], sig[9], G, h);
    } else {
        if (cs_row)
            uni_rows_diff_cs<K>(prm, xs, cs_row[0], cs_row[1], u, mu, sig, G, h);
        else
            uni_rows_diff<K>(prm, xs, u, mu, sig, G, h);
    }
}

// What one env's CBFQPLayer forward leaves behind (the backward re-uses it).
template <int MODE, int K>
struct LayerState {
    using D = Dims<MODE, K>;
    float G[D::M][D::N];  // normalised rows (what qpth sees)
    float h[D::M];
    float Graw[D::M][D::N];
    float hraw[D::M];
    float Nrm[D::M];
    bool ish[D::M];
    QPResult<D::N, D::M> qp;
};

// CBFQPLayer.get_safe_action for one env (diff_cbf_qp.py:44-79):
// build -> normalise -> fp64 QP -> .float() -> clamp.
// NEED_LAM: the caller needs the multipliers and the active set (backward);
// otherwise the cars path uses the 1-D exact solver (cars_qp_1d).
// RAW (the fused safe step, exact solver only): the rows are solved as built,
// without the row normalisation -- a positive scaling of each row that the
// exact optimum does not depend on (cars_qp_1d_raw); L.G / L.h then hold the
// raw rows and L.Nrm / L.ish are not set.
// The exact solve of the RAW rows (the fused safe step's layer, after the
// rows are built): P of the diff layer, the closed-form solver of the mode,
// then u_final = clamp(u + z[:n_u]) (diff_cbf_qp.py:77).  Shared by
// layer_forward<..., RAW> and the cars early-store order in k_safe_step.
template <int MODE, int K>
__device__ __forceinline__ void layer_solve_raw(const rcbf_params& prm, const float* u, float* u_final,
                                                LayerState<MODE, K>& L) {
    using D = Dims<MODE, K>;
    PMat<D::N, true> pm;
    double pd[D::N];
    diff_P<MODE>(pd);
    pmat_set_diag<D::N>(pm, pd);
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS)
        cars_qp_1d_raw<float>(pm, L.G, L.h, L.qp.z, L.qp.status);
    else
        uni_qp_2d_raw<K, float>(pm, L.G, L.h, L.qp.z, L.qp.status);
#pragma unroll
    for (int c = 0; c < D::NU; ++c) {
        float v = u[c] + (float)L.qp.z[c];
        float lo = (float)prm.u_min[c], hi = (float)prm.u_max[c];
        u_final[c] = fminf(fmaxf(v, lo), hi);  // torch.clamp (diff_cbf_qp.py:77)
    }
}

template <int SOLVER, int MODE, int K, bool NEED_LAM = false, bool ST = false, bool RAW = false>
__device__ __forceinline__ void layer_forward(const rcbf_params& prm, const float* xs, const float* u,
                                              const float* mu, const float* sig, float* u_final,
                                              LayerState<MODE, K>& L, const Stamps<ST>& stamps = {},
                                              const float* cs_row = nullptr) {
    using D = Dims<MODE, K>;
    diff_rows<MODE, K>(prm, xs, u, mu, sig, L.G, L.h, cs_row);
    if constexpr (RAW && SOLVER == RCBF_SOLVER_ACTIVE_SET && !NEED_LAM) {
        stamps.mark(3, false);
        layer_solve_raw<MODE, K>(prm, u, u_final, L);
        stamps.mark(4, false);
        return;
    }
#pragma unroll
    for (int r = 0; r < D::M; ++r) {
        L.hraw[r] = L.h[r];
#pragma unroll
        for (int k = 0; k < D::N; ++k) L.Graw[r][k] = L.G[r][k];
    }
    normalize_layer_rows<D::N, D::M, 2 * D::NU>(L.G, L.h, L.Nrm, L.ish);
    stamps.mark(3, false);
    PMat<D::N, true> pm;
    double pd[D::N], q[D::N];
    diff_P<MODE>(pd);
#pragma unroll
    for (int k = 0; k < D::N; ++k) q[k] = 0.0;
    pmat_set_diag<D::N>(pm, pd);
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS && SOLVER == RCBF_SOLVER_ACTIVE_SET && !NEED_LAM) {
        cars_qp_1d<float>(pm, L.G, L.h, L.qp.z, L.qp.status);
    } else if constexpr (MODE == RCBF_MODE_UNICYCLE && SOLVER == RCBF_SOLVER_ACTIVE_SET && !NEED_LAM) {
        uni_qp_2d<K, float>(pm, L.G, L.h, L.qp.z, L.qp.status);
    } else {
        qp_solve<SOLVER, D::N, D::M, true, float>(pm, q, L.G, L.h, prm.max_iter, prm.eps, L.qp);
    }
    stamps.mark(4, false);
#pragma unroll
    for (int c = 0; c < D::NU; ++c) {
        float v = u[c] + (float)L.qp.z[c];
        float lo = (float)prm.u_min[c], hi = (float)prm.u_max[c];
        u_final[c] = fminf(fmaxf(v, lo), hi);  // torch.clamp (diff_cbf_qp.py:77)
    }
}

__device__ __forceinline__ void report(int status, int32_t* status_out, int64_t i, int32_t* fail_flag) {
    if (status_out) status_out[i] = status;
    if (status != RCBF_QP_OK && fail_flag) atomicOr(fail_flag, 1 << status);
}

// ---------------------------------------------------------------------------
// environments
// ---------------------------------------------------------------------------
// Env state in HBM is component-PAIR-major: components (2p, 2p+1) of env i
// sit at x[2 (p B + i)] and x[2 (p B + i) + 1] (a (B, 2) block per pair), and
// an odd last component n_s-1 at x[(n_s-1) B + i].  Every lane moves 16 B per
// pair, so a wavefront's pair load/store is one contiguous 1 KiB dwordx4
// access (half the memory instructions of plain SoA).  For B = 1 the layout
// is the state row itself.  aux/step/episode are (B,) vectors.
template <int MODE>
__device__ __forceinline__ void env_reset_one(const double* noise, int64_t i, uint64_t seed, int64_t off,
                                              uint32_t ep, double* xs, double& aux, int& st) {
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        double nz = noise ? noise[i] : 0.5 * normal_draw(seed, (uint64_t)(off + i), ep);
        cars_reset_state(xs, nz);
        aux = 0.0;
    } else {
        uni_reset_state(xs, aux);
    }
    st = 0;
}

template <int MODE>
__device__ __forceinline__ void env_obs(const double* xs, double* o) {
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        cars_obs(xs, o);
    } else {
        uni_obs(xs, o);
    }
}

// DynamicsModel.get_state (dynamics.py:190-232) on an fp32 observation row:
// cars scale positions x100, velocities x30 (numpy fp32 in-place multiply:
// one rounding of the exact product, which the fp64 product then cast
// reproduces); unicycle theta = arctan2(sin, cos).  Result cast to fp32 like
// to_tensor(state, obs.dtype).
template <int MODE>
__device__ __forceinline__ void state_from_obs32(const float* o, float* s32) {
#pragma clang fp contract(off)
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
#pragma unroll
        for (int k = 0; k < 10; ++k) s32[k] = (float)((double)o[k] * ((k & 1) ? 30.0 : 100.0));
    } else {
        s32[0] = o[0];
        s32[1] = o[1];
        s32[2] = (float)atan2((double)o[3], (double)o[2]);
    }
}

// state32 = get_state(float(obs(x)))   (dynamics.py:190-232, via the fp32
// observation the policy sees: sac_cbf.py:61 then to_numpy/fp64/rescale/fp32)
template <int MODE>
__device__ __forceinline__ void state_from_env(const double* xs, float* s32) {
    double o[Dims<MODE, 1>::NO];
    env_obs<MODE>(xs, o);
    float o32[Dims<MODE, 1>::NO];
#pragma unroll
    for (int k = 0; k < Dims<MODE, 1>::NO; ++k) o32[k] = (float)o[k];
    state_from_obs32<MODE>(o32, s32);
}

// One fused safe step for one env (shared by k_safe_step and k_safe_rollout).
// The episode counter is only touched when the env resets.
// obs_cache (unicycle): cos/sin/goal distance of the post-step state, valid
// unless the env was reset (then obs_cache[3] = 0 and the obs is recomputed).
template <int SOLVER, int MODE, int K, bool ST = false, bool WT = false>
__device__ __forceinline__ void safe_step_one(const rcbf_params& prm, int64_t i, double* xs, double& a, int& st,
                                              uint32_t* episode, const float* us, const float* m, const float* s,
                                              float* uf, float& rew, float& cst, bool& dn, bool& gm, int& status,
                                              int auto_reset, uint64_t seed, int64_t off,
                                              const Stamps<ST>& stamps = {}, double* obs_cache = nullptr,
                                              bool ep_pre = false, uint32_t ep0 = 0) {
    using D = Dims<MODE, K>;
    float s32[D::NS];
    float cs_row[2];
    double c_th = 0.0, s_th = 0.0;  // unicycle: cos/sin of the pre-step theta, shared by obs, rows and env step
    if constexpr (MODE == RCBF_MODE_UNICYCLE) {
#ifndef RCBF_STUDY_UNI_NO_SINCOS
        sincos(xs[2], &s_th, &c_th);
#else  // study build, timing only (results invalid): the pre-step sincos replaced by a cheap stand-in
        c_th = fma(-0.5 * xs[2], xs[2], 1.0);
        s_th = xs[2];
#endif
        uni_state32_from_cs(xs, c_th, s_th, s32, cs_row[0], cs_row[1]);
    } else {
        state_from_env<MODE>(xs, s32);
    }
    stamps.mark(2, false);
    LayerState<MODE, K> L;
    layer_forward<SOLVER, MODE, K, false, ST, RCBF_FUSED_RAW_ROWS != 0>(prm, s32, us, m, s, uf, L, stamps,
                                                                       MODE == RCBF_MODE_UNICYCLE ? cs_row : nullptr);
    status = L.qp.status;
    stamps.count(9, uf[0] != us[0]);  // lanes whose action the filter changed
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        CarsStepOut o;
        cars_env_step<float>(prm, xs, a, st, uf[0], o);
        rew = o.reward;
        cst = (float)o.cost;
        dn = o.done;
        gm = false;
    } else {
        UniStepOut o;
        uni_env_step_cs<float, K>(prm, xs, a, st, uf, c_th, s_th, o);
        rew = (float)o.reward;
        cst = (float)o.cost;
        dn = o.done;
        gm = o.goal;
        if (obs_cache) {
            obs_cache[0] = o.c;
            obs_cache[1] = o.s;
            obs_cache[2] = o.gd;
            obs_cache[3] = 1.0;
        }
    }
    stamps.mark(5, false);
    if (auto_reset && dn) {
        // ep_pre: the caller loaded episode[i] with the state (reset_foreseeable)
        uint32_t ep = episode ? (ep_pre ? ep0 : episode[i]) + 1u : 0u;
        if (episode) {
            if constexpr (WT)
                st_wt(&episode[i], ep);
            else
                episode[i] = ep;
        }
        env_reset_one<MODE>(nullptr, i, seed, off, ep, xs, a, st);
        if (obs_cache) {
            if constexpr (MODE == RCBF_MODE_UNICYCLE) {  // the reset state's obs inputs
                obs_cache[0] = 1.0;                       // cos 0
                obs_cache[1] = 0.0;                       // sin 0
                obs_cache[2] = a;                         // goal distance of the reset state
                obs_cache[3] = 1.0;
            } else {
                obs_cache[3] = 0.0;
            }
        }
    }
}

// Whether this env can finish its episode in this step, known before the
// step: the time limit, or (unicycle) being within reach of the goal (a step
// moves the robot by at most dt (|u0| + 0.1) = 0.022 < 0.2 and the goal test
// is d <= 0.3).  Such envs load their episode counter together with the state
// so the reset does not wait on a dependent load at the end of the step.
template <int MODE>
__device__ __forceinline__ bool reset_foreseeable(int st, double aux) {
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS)
        return st + 1 >= 300;
    else
        return st + 1 >= 1000 || aux <= 0.5;
}

inline int check_prm(const rcbf_params* prm) {
    if (!prm) return RCBF_E_NULL;
    if (prm->mode != RCBF_MODE_SIMULATED_CARS && prm->mode != RCBF_MODE_UNICYCLE) return RCBF_E_BAD_MODE;
    if (prm->mode == RCBF_MODE_UNICYCLE && (prm->num_hazards < 1 || prm->num_hazards > RCBF_MAX_HAZARDS))
        return RCBF_E_BAD_SHAPE;
    if (prm->solver != RCBF_SOLVER_ACTIVE_SET && prm->solver != RCBF_SOLVER_PDIPM && prm->solver != RCBF_SOLVER_GI)
        return RCBF_E_BAD_MODE;
    return 0;
}

inline int launch_status() { return (int)hipGetLastError(); }

}  // namespace rcbf

// Launch KERNEL (a template-id naming BS_) over B envs at the workgroup size
// block_for_envs(B): BS_ is 256, 128 or 64 in the three instantiations.
#define RCBF_BS_LAUNCH(B, KERNEL, stream, ...)                                                                \
    do {                                                                                                    \
        const int bs_ = rcbf::block_for_envs(B);                                                            \
        if (bs_ == 256) {                                                                                   \
            constexpr int BS_ = 256;                                                                        \
            hipLaunchKernelGGL(KERNEL, dim3(rcbf::grid_for_envs(B, BS_)), dim3(BS_), 0, stream, __VA_ARGS__); \
        } else if (bs_ == 128) {                                                                            \
            constexpr int BS_ = 128;                                                                        \
            hipLaunchKernelGGL(KERNEL, dim3(rcbf::grid_for_envs(B, BS_)), dim3(BS_), 0, stream, __VA_ARGS__); \
        } else {                                                                                            \
            constexpr int BS_ = 64;                                                                         \
            hipLaunchKernelGGL(KERNEL, dim3(rcbf::grid_for_envs(B, BS_)), dim3(BS_), 0, stream, __VA_ARGS__); \
        }                                                                                                   \
    } while (0)

// The same for a kernel instantiated per solver: only the exact (default)
// solver gets the small workgroups; the others always run 256-thread ones (in
// the small branches BS_ folds to 256 for them, so no extra instantiation).
#define RCBF_BS_LAUNCH_S(SOLVER, B, KERNEL, stream, ...)                                                      \
    do {                                                                                                    \
        constexpr bool exact_ = (SOLVER) == RCBF_SOLVER_ACTIVE_SET;                                         \
        const int bs_ = exact_ ? rcbf::block_for_envs(B) : 256;                                             \
        if (bs_ == 256) {                                                                                   \
            constexpr int BS_ = 256;                                                                        \
            hipLaunchKernelGGL(KERNEL, dim3(rcbf::grid_for_envs(B, BS_)), dim3(BS_), 0, stream, __VA_ARGS__); \
        } else if (bs_ == 128) {                                                                            \
            constexpr int BS_ = exact_ ? 128 : 256;                                                         \
            hipLaunchKernelGGL(KERNEL, dim3(rcbf::grid_for_envs(B, BS_)), dim3(BS_), 0, stream, __VA_ARGS__); \
        } else {                                                                                            \
            constexpr int BS_ = exact_ ? 64 : 256;                                                          \
            hipLaunchKernelGGL(KERNEL, dim3(rcbf::grid_for_envs(B, BS_)), dim3(BS_), 0, stream, __VA_ARGS__); \
        }                                                                                                   \
    } while (0)

// Dispatch a launch over (mode, unicycle hazard count) -> MODE_, K_.
#define RCBF_DISPATCH_MODE(prm, ...)                                 \
    do {                                                             \
        if ((prm)->mode == RCBF_MODE_SIMULATED_CARS) {               \
            constexpr int MODE_ = RCBF_MODE_SIMULATED_CARS;          \
            constexpr int K_ = 1;                                    \
            __VA_ARGS__;                                             \
        } else {                                                     \
            constexpr int MODE_ = RCBF_MODE_UNICYCLE;                \
            switch ((prm)->num_hazards) {                            \
                case 1: { constexpr int K_ = 1; __VA_ARGS__; } break; \
                case 2: { constexpr int K_ = 2; __VA_ARGS__; } break; \
                case 3: { constexpr int K_ = 3; __VA_ARGS__; } break; \
                case 4: { constexpr int K_ = 4; __VA_ARGS__; } break; \
                case 5: { constexpr int K_ = 5; __VA_ARGS__; } break; \
                case 6: { constexpr int K_ = 6; __VA_ARGS__; } break; \
                case 7: { constexpr int K_ = 7; __VA_ARGS__; } break; \
                default: { constexpr int K_ = 8; __VA_ARGS__; } break; \
            }                                                        \
        }                                                            \
    } while (0)

// ... and over the solver -> SOLVER_.
#define RCBF_DISPATCH(prm, ...)                                                        \
    do {                                                                               \
        if ((prm)->solver == RCBF_SOLVER_PDIPM) {                                      \
            constexpr int SOLVER_ = RCBF_SOLVER_PDIPM;                                 \
            RCBF_DISPATCH_MODE(prm, __VA_ARGS__);                                      \
        } else if ((prm)->solver == RCBF_SOLVER_GI) {                                  \
            constexpr int SOLVER_ = RCBF_SOLVER_GI;                                    \
            RCBF_DISPATCH_MODE(prm, __VA_ARGS__);                                      \
        } else {                                                                       \
            constexpr int SOLVER_ = RCBF_SOLVER_ACTIVE_SET;                            \
            RCBF_DISPATCH_MODE(prm, __VA_ARGS__);                                      \
        }                                                                              \
    } while (0)
