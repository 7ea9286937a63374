// rcbf_model.hip -- model-based rollout step and the
// device replay buffer's ring scatter / row gather (8f row 4) + C-ABI.
//
// rcbf_model_step restates one k-step of generate_model_rollouts
// (rcbf_sac/generate_rollouts.py:24-77) for a batch of replay transitions:
//   state = get_state(obs); (mu, std) = predict_next_state(state, a, t)
//   (model prior + dt * disturbance mean, dt * disturbance std);
//   next_state = mu + std * z; next_obs = get_obs(next_state) (+ compass and
//   exp(-dist) for the unicycle); reward, done -> mask; next_t = t + dt.
// All fp64 like the reference's numpy, with FMA contraction off so the
// products round as numpy's do.
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// The workgroup's rows (W elements of T each, row-major, rows row0 .. row0 + nrows) through LDS, so the
// global accesses are whole coalesced 16-B lane vectors; a row per lane would put the lanes W sizeof(T)
// bytes apart, each of its W load instructions touching a line per 1-2 lanes.  16-B accesses when the block's first element is 16-B aligned (a tensor's own storage is;
// a sliced view may not be), element accesses otherwise; all of a thread's loads are issued before its
// LDS stores.  s: kBlock * W elements, 16-B aligned.
template <typename T, int W>
__device__ __forceinline__ void rows_in(const T* __restrict__ src, int64_t row0, int nrows, T* s) {
    constexpr int V = 16 / (int)sizeof(T);
    const T* p = src + row0 * W;
    const int n = nrows * W, t = threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        constexpr int kIt = (kBlock * W / V + kBlock - 1) / kBlock;
        const int nv = n / V;
        u32x4 v[kIt];
#pragma unroll
        for (int j = 0; j < kIt; ++j) {
            const int e = t + j * kBlock;
            if (e < nv) v[j] = reinterpret_cast<const u32x4*>(p)[e];
        }
#pragma unroll
        for (int j = 0; j < kIt; ++j) {
            const int e = t + j * kBlock;
            if (e < nv) reinterpret_cast<u32x4*>(s)[e] = v[j];
        }
        if (t < n - nv * V) s[nv * V + t] = p[nv * V + t];
    } else {
        T v[W];
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int e = t + j * kBlock;
            if (e < n) v[j] = p[e];
        }
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int e = t + j * kBlock;
            if (e < n) s[e] = v[j];
        }
    }
}

template <typename T, int W>
__device__ __forceinline__ void rows_out(T* __restrict__ dst, int64_t row0, int nrows, const T* s) {
    constexpr int V = 16 / (int)sizeof(T);
    T* p = dst + row0 * W;
    const int n = nrows * W, t = threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        constexpr int kIt = (kBlock * W / V + kBlock - 1) / kBlock;
        const int nv = n / V;
#pragma unroll
        for (int j = 0; j < kIt; ++j) {
            const int e = t + j * kBlock;
            if (e < nv) reinterpret_cast<u32x4*>(p)[e] = reinterpret_cast<const u32x4*>(s)[e];
        }
        if (t < n - nv * V) p[nv * V + t] = s[nv * V + t];
    } else {
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int e = t + j * kBlock;
            if (e < n) p[e] = s[e];
        }
    }
}

// get_state (dynamics.py:190-232), numpy fp64 path
template <int MODE>
__device__ __forceinline__ void model_state_from_obs(const double* o, double* xs) {
#pragma clang fp contract(off)
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
#pragma unroll
        for (int k = 0; k < 10; ++k) xs[k] = o[k] * ((k & 1) ? 30.0 : 100.0);
    } else {
        xs[0] = o[0];
        xs[1] = o[1];
        xs[2] = atan2(o[3], o[2]);
    }
}

// x + dt (f(x) + g(x) u) of the model prior (dynamics.py:60-105, 125-188)
template <int MODE>
__device__ __forceinline__ void model_prior_next(const double* xs, const double* u, double t, double* nx) {
#pragma clang fp contract(off)
    const double dt = 0.02;
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        double pos[5], vel[5], acc[5];
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            pos[c] = xs[2 * c];
            vel[c] = xs[2 * c + 1];
        }
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            double vdes = 30.0;
            if (c == 0) vdes -= 10.0 * sin(0.2 * t);
            acc[c] = 4.0 * (vdes - vel[c]);
        }
        const double d01 = pos[0] - pos[1], d12 = pos[1] - pos[2], d24 = pos[2] - pos[4];
        acc[1] -= 20.0 * d01 * (d01 < 6.0 ? 1.0 : 0.0);
        acc[2] -= 20.0 * d12 * (d12 < 6.0 ? 1.0 : 0.0);
        acc[3] = 0.0;
        acc[4] -= 20.0 * d24 * (d24 < 13.0 ? 1.0 : 0.0);
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            nx[2 * c] = xs[2 * c] + dt * (vel[c] + 0.0);
            nx[2 * c + 1] = xs[2 * c + 1] + dt * (acc[c] + (c == 3 ? 50.0 * u[0] : 0.0));
        }
    } else {
        double s, c;
        sincos(xs[2], &s, &c);
        nx[0] = xs[0] + dt * (0.0 + c * u[0]);
        nx[1] = xs[1] + dt * (0.0 + s * u[0]);
        nx[2] = xs[2] + dt * (0.0 + u[1]);
    }
}

template <int MODE>
__global__ void __launch_bounds__(kBlock) k_model_step(rcbf_params prm, int64_t B, const double* __restrict__ obs,
                                                       const double* __restrict__ act, const double* __restrict__ t,
                                                       const float* __restrict__ mean, const float* __restrict__ stdv,
                                                       const double* __restrict__ z, uint64_t seed, uint64_t counter,
                                                       double* __restrict__ next_obs, double* __restrict__ reward,
                                                       double* __restrict__ mask, double* __restrict__ next_t) {
#pragma clang fp contract(off)
    using D = Dims<MODE, 1>;
    constexpr int NS = D::NS, NO = D::NO, NU = D::NU;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    const double dt = 0.02;
    double o[NO], xs[NS], u[NU], nx[NS];
#pragma unroll
    for (int k = 0; k < NO; ++k) o[k] = obs[i * NO + k];
#pragma unroll
    for (int c = 0; c < NU; ++c) u[c] = act[i * NU + c];
    const double ti = t ? t[i] : 0.0;
    model_state_from_obs<MODE>(o, xs);
    model_prior_next<MODE>(xs, u, ti, nx);
    // disturbance: GP (mean, std) or the zero-mean MAX_STD prior (dynamics.py:381-384)
    double zz[NS];
    if (z) {
#pragma unroll
        for (int k = 0; k < NS; ++k) zz[k] = z[i * NS + k];
    } else {  // N(0,1) from Philox4x32-10 keyed by (seed, row, counter, call q): one call = 4 words = 2
              // Box-Muller pairs on 24-bit uniforms with the hardware fp32 log2 / sin / cos (as the envs'
              // reset draw, normal_draw); statistically N(0, 1), |z| <= 5.8 (r04: cars 5 fp64 pairs -> 3 calls)
#pragma unroll
        for (int q = 0; q < (NS + 3) / 4; ++q) {
            uint32_t cc[4] = {(uint32_t)i, (uint32_t)((uint64_t)i >> 32), (uint32_t)counter, (uint32_t)q};
            philox4x32_10(cc, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float f1 = ((float)(cc[2 * h] >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
                const float f2 = (float)(cc[2 * h + 1] >> 8) * (1.0f / 16777216.0f);      // [0, 1) revolutions
                const float r = __builtin_sqrtf(-2.0f * __builtin_amdgcn_logf(f1) * 0.69314718f);
                const int k = 4 * q + 2 * h;
                if (k < NS) zz[k] = (double)(r * __builtin_amdgcn_cosf(f2));
                if (k + 1 < NS) zz[k + 1] = (double)(r * __builtin_amdgcn_sinf(f2));
            }
        }
    }
    double ns[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const double m = mean ? (double)mean[i * NS + k] : 0.0;
        // MAX_STD as numpy fp64 (dynamics.py:24,381-384)
        const double prior = (MODE == RCBF_MODE_UNICYCLE || (k & 1)) ? 0.2 : 0.0;
        const double sd = stdv ? (double)stdv[i * NS + k] : prior;
        const double mu = nx[k] + dt * m;      // next_state_batch += dt * pred_mean
        ns[k] = mu + (dt * sd) * zz[k];        // np.random.normal(mu, dt * pred_std)
    }
    double r, msk;
    const double tn = ti + dt;
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
#pragma unroll
        for (int k = 0; k < 10; ++k)  // correctly rounded x / d in 3 FMAs (div_const), numpy's x / d bit for bit
            next_obs[i * NO + k] = (k & 1) ? div_const(ns[k], 30.0, 1.0 / 30.0) : div_const(ns[k], 100.0, 1.0 / 100.0);
        r = -5.0 * fabs(u[0] * u[0]) / 300.0;     // generate_rollouts.py:62
        msk = (tn >= 300.0 * 0.02) ? 0.0 : 1.0;   // :65-66
    } else {
        double s, c;
        sincos(ns[2], &s, &c);
        const double g0 = 2.5 - ns[0], g1 = 2.5 - ns[1];
        const double d = sqrt(g0 * g0 + g1 * g1);
        double c0 = g0 * c + g1 * s;       // goal_rel @ R(theta)  (:41)
        double c1 = g0 * (-s) + g1 * c;
        const double nrm = sqrt(c0 * c0 + c1 * c1) + 0.001;
        c0 = c0 / nrm;
        c1 = c1 / nrm;
        double* nw = &next_obs[i * NO];
        nw[0] = ns[0];
        nw[1] = ns[1];
        nw[2] = c;
        nw[3] = s;
        nw[4] = c0;
        nw[5] = c1;
        nw[6] = exp(-d);
        const double dprev = -log(o[NO - 1]);
        const bool goal = d <= 0.3;
        r = (dprev - d) * 1.0 + (goal ? 1.0 : 0.0);  // :47
        r = r + 1.0 * (goal ? 1.0 : 0.0);          // :51, the goal bonus counted twice
        msk = goal ? 0.0 : 1.0;
    }
    reward[i] = r;
    mask[i] = msk;
    if (next_t) next_t[i] = tn;
}

// DynamicsModel.predict_next_state (dynamics.py:60-105) on device rows:
// next = x + dt (f(x) + g(x) u) [+ dt * mean when use_gps], std_out = dt * std
// (zeros without use_gps), next_t = t + dt.  The disturbance (mean, std) is
// the fitted GP's posterior (f32, rcbf_gp_predict) or, when null, the
// zero-mean MAX_STD prior (dynamics.py:381-384).  fp64 rows, contraction off:
// the same roundings as the reference's numpy.
template <int MODE>
__global__ void __launch_bounds__(kBlock) k_predict_next_state(int64_t B, const double* __restrict__ x,
                                                               const double* __restrict__ act,
                                                               const double* __restrict__ t,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ stdv, int use_gps,
                                                               double* __restrict__ next_x,
                                                               double* __restrict__ std_out,
                                                               double* __restrict__ next_t) {
#pragma clang fp contract(off)
    using D = Dims<MODE, 1>;
    constexpr int NS = D::NS, NU = D::NU;
    // the cars' 80-B rows (x in; next_x, std_out out; 40-B mean / std in) go through LDS (rows_in /
    // rows_out): 11.1 -> 8.0 us at B = 65 536 (r05zb); the unicycle's 24-B rows stay per lane (3.8 us
    // per lane, 4.0 staged), as do the model step's rows (6.2 us per lane, 6.4 staged: its time is the
    // fp64 sin / Philox chain, not the access pattern)
    constexpr bool kStage = NS * (int)sizeof(double) >= 64;
    constexpr int kS = kStage ? kBlock * NS / 2 + 1 : 1, kM = kStage ? kBlock * NS / 4 + 1 : 1;
    __shared__ u32x4 s_x[kS], s_sd[kS], s_ms[2][kM];
    double* sx = reinterpret_cast<double*>(s_x);
    double* sd_rows = reinterpret_cast<double*>(s_sd);
    const int64_t row0 = (int64_t)blockIdx.x * kBlock;
    const int nrows = (int)min((int64_t)kBlock, B - row0);
    const int64_t i = row0 + threadIdx.x;
    const bool live = threadIdx.x < nrows;
    if constexpr (!kStage) {
        if (!live) return;
    } else {
        rows_in<double, NS>(x, row0, nrows, sx);
        if (use_gps && mean) rows_in<float, NS>(mean, row0, nrows, reinterpret_cast<float*>(s_ms[0]));
        if (use_gps && stdv) rows_in<float, NS>(stdv, row0, nrows, reinterpret_cast<float*>(s_ms[1]));
    }
    const double dt = 0.02;
    double xs[NS], u[NU], nx[NS];
#pragma unroll
    for (int c = 0; c < NU; ++c) u[c] = live ? act[i * NU + c] : 0.0;
    const double ti = (t && live) ? t[i] : 0.0;
    if constexpr (kStage) __syncthreads();
#pragma unroll
    for (int k = 0; k < NS; ++k) xs[k] = kStage ? sx[threadIdx.x * NS + k] : x[i * NS + k];
    model_prior_next<MODE>(xs, u, ti, nx);
    const float* sm = kStage ? reinterpret_cast<const float*>(s_ms[0]) + threadIdx.x * NS : mean + i * NS;
    const float* ss = kStage ? reinterpret_cast<const float*>(s_ms[1]) + threadIdx.x * NS : stdv + i * NS;
    if constexpr (kStage) __syncthreads();  // every thread has read its x row: the buffer takes the next_x rows
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        double sd = 0.0;
        if (use_gps) {
            const double m = mean ? (double)sm[k] : 0.0;
            const double prior = (MODE == RCBF_MODE_UNICYCLE || (k & 1)) ? 0.2 : 0.0;  // MAX_STD
            sd = stdv ? (double)ss[k] : prior;
            nx[k] = nx[k] + dt * m;  // next_state_batch += dt * pred_mean
        }
        if constexpr (kStage) {
            sx[threadIdx.x * NS + k] = nx[k];
            sd_rows[threadIdx.x * NS + k] = dt * sd;
        } else {
            next_x[i * NS + k] = nx[k];
            std_out[i * NS + k] = dt * sd;
        }
    }
    if (next_t && live) next_t[i] = ti + dt;
    if constexpr (kStage) {
        __syncthreads();
        rows_out<double, NS>(next_x, row0, nrows, sx);
        rows_out<double, NS>(std_out, row0, nrows, sd_rows);
    }
}

// Replay ring (rcbf_sac/replay_memory.py:12-32): records are rows of W f64.
__global__ void __launch_bounds__(256) k_ring_scatter(double* __restrict__ ring, int64_t cap, int64_t W, int64_t pos,
                                                      const double* __restrict__ src, int64_t n) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n * W) return;
    const int64_t r = e / W, c = e - r * W;
    ring[((pos + r) % cap) * W + c] = src[e];
}

__global__ void __launch_bounds__(256) k_gather_rows(double* __restrict__ dst, const double* __restrict__ ring,
                                                     int64_t W, const int64_t* __restrict__ idx, int64_t n) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n * W) return;
    const int64_t r = e / W, c = e - r * W;
    dst[e] = ring[idx[r] * W + c];
}

}  // namespace

// DynamicsModel.get_state on fp32 observation rows (dynamics.py:190-232): the
// state rcbf_obs_safe_action forms in-kernel (state_from_obs32), one row per thread
template <int MODE>
__global__ void __launch_bounds__(kBlock) k_state_from_obs(int64_t B, const float* __restrict__ obs,
                                                           float* __restrict__ state) {
    using D = Dims<MODE, 1>;
    const int64_t i = env_index();
    if (i >= B) return;
    float o[D::NO], s32[D::NS];
#pragma unroll
    for (int k = 0; k < D::NO; ++k) o[k] = obs[i * D::NO + k];
    state_from_obs32<MODE>(o, s32);
#pragma unroll
    for (int k = 0; k < D::NS; ++k) state[i * D::NS + k] = s32[k];
}

extern "C" {

int rcbf_model_step(const rcbf_params* prm, int64_t B, const double* obs, const double* act, const double* t,
                    const float* mean, const float* stdv, const double* z, uint64_t seed, uint64_t counter,
                    double* next_obs, double* reward, double* mask, double* next_t, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!obs || !act || !next_obs || !reward || !mask) return RCBF_E_NULL;
    if (prm->mode == RCBF_MODE_SIMULATED_CARS && !t) return RCBF_E_NULL;  // cars dynamics need t
    dim3 g(grid_for(B)), b(kBlock);
    if (prm->mode == RCBF_MODE_SIMULATED_CARS)
        hipLaunchKernelGGL((k_model_step<RCBF_MODE_SIMULATED_CARS>), g, b, 0, stream, *prm, B, obs, act, t, mean, stdv,
                           z, seed, counter, next_obs, reward, mask, next_t);
    else
        hipLaunchKernelGGL((k_model_step<RCBF_MODE_UNICYCLE>), g, b, 0, stream, *prm, B, obs, act, t, mean, stdv, z,
                           seed, counter, next_obs, reward, mask, next_t);
    return launch_status();
}

int rcbf_predict_next_state(const rcbf_params* prm, int64_t B, const double* x, const double* act, const double* t,
                            const float* mean, const float* stdv, int32_t use_gps, double* next_x, double* std_out,
                            double* next_t, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !act || !next_x || !std_out) return RCBF_E_NULL;
    if (prm->mode == RCBF_MODE_SIMULATED_CARS && !t) return RCBF_E_NULL;  // cars dynamics need t
    if (next_t && !t) return RCBF_E_NULL;
    dim3 g(grid_for(B)), b(kBlock);
    if (prm->mode == RCBF_MODE_SIMULATED_CARS)
        hipLaunchKernelGGL((k_predict_next_state<RCBF_MODE_SIMULATED_CARS>), g, b, 0, stream, B, x, act, t, mean,
                           stdv, (int)use_gps, next_x, std_out, next_t);
    else
        hipLaunchKernelGGL((k_predict_next_state<RCBF_MODE_UNICYCLE>), g, b, 0, stream, B, x, act, t, mean, stdv,
                           (int)use_gps, next_x, std_out, next_t);
    return launch_status();
}

int rcbf_state_from_obs(const rcbf_params* prm, int64_t B, const float* obs, float* state_out, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!obs || !state_out) return RCBF_E_NULL;
    if (prm->mode == RCBF_MODE_SIMULATED_CARS)
        hipLaunchKernelGGL((k_state_from_obs<RCBF_MODE_SIMULATED_CARS>), dim3(grid_for(B)), dim3(kBlock), 0, stream, B,
                           obs, state_out);
    else
        hipLaunchKernelGGL((k_state_from_obs<RCBF_MODE_UNICYCLE>), dim3(grid_for(B)), dim3(kBlock), 0, stream, B, obs,
                           state_out);
    return launch_status();
}

int rcbf_ring_scatter_f64(double* ring, int64_t cap, int64_t W, int64_t pos, const double* src, int64_t n,
                          hipStream_t stream) {
    if (cap < 1 || W < 1 || n < 0 || pos < 0 || n > cap) return RCBF_E_BAD_SHAPE;
    if (n == 0) return 0;
    if (!ring || !src) return RCBF_E_NULL;
    hipLaunchKernelGGL(k_ring_scatter, dim3((unsigned)((n * W + 255) / 256)), dim3(256), 0, stream, ring, cap, W,
                       pos % cap, src, n);
    return launch_status();
}

int rcbf_gather_rows_f64(double* dst, const double* ring, int64_t W, const int64_t* idx, int64_t n,
                         hipStream_t stream) {
    if (W < 1 || n < 0) return RCBF_E_BAD_SHAPE;
    if (n == 0) return 0;
    if (!dst || !ring || !idx) return RCBF_E_NULL;
    hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((n * W + 255) / 256)), dim3(256), 0, stream, dst, ring, W, idx,
                       n);
    return launch_status();
}

}  // extern "C"
