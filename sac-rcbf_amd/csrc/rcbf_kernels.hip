// rcbf_kernels.hip -- gfx950 kernels + C-ABI of librcbf_hip.so (include/rcbf_hip.h).
//
// Every kernel maps one env (or one QP) to one lane of a 64-wide wavefront,
// 256-thread workgroups.  The env / CBF / QP state of a lane never leaves
// VGPRs inside a launch; HBM sees each input byte once and each output byte
// once (the fused step reads x, t, step, u_RL and writes x', t', step', obs,
// u, reward, cost, done).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "rcbf_device.hpp"

using namespace rcbf;

namespace {

#ifndef RCBF_BLOCK
#define RCBF_BLOCK 256
#endif
constexpr int kBlock = RCBF_BLOCK;
// Ablation switches for performance studies only (scripts/ablate.sh builds
// them into separate libraries; the product build uses 0):
//   1 = no QP (u_qp = 0), 2 = no rows/normalise/QP, 4 = no env dynamics,
//   8 = no observation maths
#ifndef RCBF_ABLATE
#define RCBF_ABLATE 0
#endif
constexpr int kAblate = RCBF_ABLATE;

inline unsigned grid_for(int64_t B) { return (unsigned)((B + kBlock - 1) / kBlock); }

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

// Rows of the diff layer for one env, from fp32 state / u / mean / sigma.
template <int MODE, int K>
__device__ __forceinline__ void diff_rows(const rcbf_params& prm, const float* xs, const float* u,
                                          const float* mu, const float* sig,
                                          float (*G)[Dims<MODE, K>::N], float* h) {
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        cars_rows_diff(prm, xs, u[0], sig[5], sig[7], sig[9], G, h);
    } else {
        uni_rows_diff<K>(prm, xs, u, mu, sig, G, h);
    }
}

// Full CBFQPLayer.get_safe_action for one env: build -> normalise -> QP ->
// .float() -> clamp.  Returns the QP result for the backward / status.
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

template <int MODE, int K>
__device__ __forceinline__ void layer_forward(const rcbf_params& prm, const float* xs, const float* u,
                                              const float* mu, const float* sig, float* u_final,
                                              LayerState<MODE, K>& L) {
    using D = Dims<MODE, K>;
    if constexpr ((kAblate & 2) != 0) {
#pragma unroll
        for (int c = 0; c < D::NU; ++c) u_final[c] = u[c] + xs[c] * 1e-30f;
        L.qp.status = RCBF_QP_OK;
        return;
    }
    diff_rows<MODE, K>(prm, xs, u, mu, sig, L.G, L.h);
#pragma unroll
    for (int r = 0; r < D::M; ++r) {
        L.hraw[r] = L.h[r];
#pragma unroll
        for (int k = 0; k < D::N; ++k) L.Graw[r][k] = L.G[r][k];
    }
    normalize_rows<D::N, D::M, float>(L.G, L.h, L.Nrm, L.ish);
    PMat<D::N, true> pm;
    double pd[D::N], q[D::N];
    diff_P<MODE>(pd);
#pragma unroll
    for (int k = 0; k < D::N; ++k) q[k] = 0.0;
    pmat_set_diag<D::N>(pm, pd);
    if constexpr ((kAblate & 1) != 0) {
#pragma unroll
        for (int k = 0; k < D::N; ++k) L.qp.z[k] = 1e-30 * (double)(L.G[0][k] + L.h[k % D::M]);
        L.qp.status = RCBF_QP_OK;
    } else {
        qp_solve<D::N, D::M, true, float>(prm.solver, pm, q, L.G, L.h, prm.max_iter, prm.eps, L.qp);
    }
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

template <int MODE>
__device__ __forceinline__ void load_f32(const float* p, int64_t i, int n, float* o) {
    for (int k = 0; k < n; ++k) o[k] = p[i * n + k];
}

// ---------------------------------------------------------------------------
// kernels: CBF-QP layer
// ---------------------------------------------------------------------------
template <int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_build(rcbf_params prm, int64_t B, const float* __restrict__ x,
                                                  const float* __restrict__ u, const float* __restrict__ mu,
                                                  const float* __restrict__ sigma, float* __restrict__ P_out,
                                                  float* __restrict__ q_out, float* __restrict__ G_out,
                                                  float* __restrict__ h_out) {
    using D = Dims<MODE, K>;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    float xs[D::NS], us[D::NU], m[D::NS], s[D::NS];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        xs[k] = x[i * D::NS + k];
        m[k] = mu ? mu[i * D::NS + k] : 0.0f;
        s[k] = sigma ? sigma[i * D::NS + k] : prior_sigma<MODE>(k);
    }
#pragma unroll
    for (int c = 0; c < D::NU; ++c) us[c] = u[i * D::NU + c];
    float G[D::M][D::N], h[D::M];
    diff_rows<MODE, K>(prm, xs, us, m, s, G, h);
#pragma unroll
    for (int r = 0; r < D::M; ++r) {
        h_out[i * D::M + r] = h[r];
#pragma unroll
        for (int k = 0; k < D::N; ++k) G_out[(i * D::M + r) * D::N + k] = G[r][k];
    }
    if (P_out) {
        double pd[D::N];
        diff_P<MODE>(pd);
#pragma unroll
        for (int a = 0; a < D::N; ++a)
#pragma unroll
            for (int b = 0; b < D::N; ++b) P_out[(i * D::N + a) * D::N + b] = (a == b) ? (float)pd[a] : 0.0f;
    }
    if (q_out) {
#pragma unroll
        for (int a = 0; a < D::N; ++a) q_out[i * D::N + a] = 0.0f;
    }
}

template <int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_build_f64(rcbf_params prm, int64_t B, const double* __restrict__ x,
                                                      const double* __restrict__ u, const double* __restrict__ mu,
                                                      const double* __restrict__ sigma, double* __restrict__ P_out,
                                                      double* __restrict__ q_out, double* __restrict__ G_out,
                                                      double* __restrict__ h_out) {
    using D = Dims<MODE, K>;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    double xs[D::NS], us[D::NU], m[D::NS], s[D::NS];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        xs[k] = x[i * D::NS + k];
        m[k] = mu ? mu[i * D::NS + k] : 0.0;
        s[k] = sigma ? sigma[i * D::NS + k] : (double)prior_sigma<MODE>(k);
    }
#pragma unroll
    for (int c = 0; c < D::NU; ++c) us[c] = u[i * D::NU + c];
    double G[D::M][D::N], h[D::M];
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS)
        cars_rows_cascade(prm, xs, us[0], G, h);
    else
        uni_rows_cascade<K>(prm, xs, us, m, s, G, h);
#pragma unroll
    for (int r = 0; r < D::M; ++r) {
        h_out[i * D::M + r] = h[r];
#pragma unroll
        for (int k = 0; k < D::N; ++k) G_out[(i * D::M + r) * D::N + k] = G[r][k];
    }
    double pd[D::N];
    cascade_P<MODE>(pd);
    if (P_out) {
#pragma unroll
        for (int a = 0; a < D::N; ++a)
#pragma unroll
            for (int b = 0; b < D::N; ++b) P_out[(i * D::N + a) * D::N + b] = (a == b) ? pd[a] : 0.0;
    }
    if (q_out) {
#pragma unroll
        for (int a = 0; a < D::N; ++a) q_out[i * D::N + a] = 0.0;
    }
}

// Generic QP (CBFQPLayer.solve_qp + cbf_layer): rows padded to MP with the
// never-active row (0 z <= 1).
template <int N, int MP>
__global__ void __launch_bounds__(kBlock) k_qp_solve(rcbf_params prm, int64_t B, int m, const float* __restrict__ P,
                                                     const float* __restrict__ q, const float* __restrict__ G,
                                                     const float* __restrict__ h, int normalize,
                                                     float* __restrict__ z_out, double* __restrict__ lam_out,
                                                     int32_t* __restrict__ status_out, int32_t* fail_flag) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    float Gl[MP][N], hl[MP], Nrm[MP];
#pragma unroll
    for (int r = 0; r < MP; ++r) {
        bool in = r < m;
#pragma unroll
        for (int k = 0; k < N; ++k) Gl[r][k] = in ? G[(i * m + r) * N + k] : 0.0f;
        hl[r] = in ? h[i * m + r] : 1.0f;
    }
    if (normalize) normalize_rows<N, MP, float>(Gl, hl, Nrm, nullptr);
    double Pin[N][N], qd[N];
#pragma unroll
    for (int a = 0; a < N; ++a) {
        qd[a] = q ? (double)q[i * N + a] : 0.0;
#pragma unroll
        for (int b = 0; b < N; ++b) Pin[a][b] = (double)P[(i * N + a) * N + b];
    }
    PMat<N, false> pm;
    pmat_set_full<N>(pm, Pin);
    QPResult<N, MP> res;
    qp_solve<N, MP, false, float>(prm.solver, pm, qd, Gl, hl, prm.max_iter, prm.eps, res);
#pragma unroll
    for (int k = 0; k < N; ++k) z_out[i * N + k] = (float)res.z[k];
    if (lam_out) {
        for (int r = 0; r < m; ++r) lam_out[i * m + r] = 0.0;
#pragma unroll
        for (int r = 0; r < MP; ++r)
            if (r < m) lam_out[i * m + r] = res.lam[r];
    }
    report(res.status, status_out, i, fail_flag);
}

template <int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_safe_action(rcbf_params prm, int64_t B, const float* __restrict__ x,
                                                        const float* __restrict__ u, const float* __restrict__ mu,
                                                        const float* __restrict__ sigma, float* __restrict__ u_out,
                                                        int32_t* __restrict__ status_out, int32_t* fail_flag) {
    using D = Dims<MODE, K>;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    float xs[D::NS], us[D::NU], m[D::NS], s[D::NS], uf[D::NU];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        xs[k] = x[i * D::NS + k];
        m[k] = mu ? mu[i * D::NS + k] : 0.0f;
        s[k] = sigma ? sigma[i * D::NS + k] : prior_sigma<MODE>(k);
    }
#pragma unroll
    for (int c = 0; c < D::NU; ++c) us[c] = u[i * D::NU + c];
    LayerState<MODE, K> L;
    layer_forward<MODE, K>(prm, xs, us, m, s, uf, L);
#pragma unroll
    for (int c = 0; c < D::NU; ++c) u_out[i * D::NU + c] = uf[c];
    report(L.qp.status, status_out, i, fail_flag);
}

// d(final)/d(u_rl) on the active set of the exact optimum (module docstring
// of include/rcbf_hip.h).  dh_r/du_c of every row is closed form:
//   CBF rows: dh/du = Lg (cars) or a_j (unicycle) = -G_raw[r][c];
//   actuator rows (u_max - u, -u_min + u): -1 / +1.
template <int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_safe_action_bwd(rcbf_params prm, int64_t B, const float* __restrict__ x,
                                                            const float* __restrict__ u, const float* __restrict__ mu,
                                                            const float* __restrict__ sigma,
                                                            const float* __restrict__ grad_u,
                                                            float* __restrict__ grad_u_rl) {
    using D = Dims<MODE, K>;
    constexpr int N = D::N, M = D::M, NU = D::NU;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    float xs[D::NS], us[NU], m[D::NS], s[D::NS], uf[NU];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        xs[k] = x[i * D::NS + k];
        m[k] = mu ? mu[i * D::NS + k] : 0.0f;
        s[k] = sigma ? sigma[i * D::NS + k] : prior_sigma<MODE>(k);
    }
#pragma unroll
    for (int c = 0; c < NU; ++c) us[c] = u[i * NU + c];
    LayerState<MODE, K> L;
    layer_forward<MODE, K>(prm, xs, us, m, s, uf, L);
    double pd[N];
    diff_P<MODE>(pd);
    // active rows (slots) from the solver
    double GA[N][N];
    int aidx[N];
    int nact = 0;
#pragma unroll
    for (int sl = 0; sl < N; ++sl) {
        aidx[sl] = -1;
#pragma unroll
        for (int k = 0; k < N; ++k) GA[sl][k] = 0.0;
    }
#pragma unroll
    for (int r = 0; r < M; ++r) {
        bool a = (L.qp.active >> r) & 1u;
#pragma unroll
        for (int sl = 0; sl < N; ++sl) {
            bool here = a && (sl == nact);
#pragma unroll
            for (int k = 0; k < N; ++k) GA[sl][k] = here ? (double)L.G[r][k] : GA[sl][k];
            aidx[sl] = here ? r : aidx[sl];
        }
        nact += a ? 1 : 0;
    }
    nact = nact > N ? N : nact;
    double J[NU][NU];  // J[i][c] = d(u_i + z_i)/d u_c
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        double dGn[M][N], dhn[M];
#pragma unroll
        for (int r = 0; r < M; ++r) {
            double dh;
            const int K0 = M - 2 * NU;  // first actuator row
            if (r < K0)
                dh = -(double)L.Graw[r][c];
            else {
                int col = (r - K0) / 2;
                bool upper = ((r - K0) % 2) == 0;
                dh = (col == c) ? (upper ? -1.0 : 1.0) : 0.0;
            }
            double hr = (double)L.hraw[r];
            double dN = L.ish[r] ? ((hr > 0.0) ? dh : ((hr < 0.0) ? -dh : 0.0)) : 0.0;
            double Nr = (double)L.Nrm[r];
            dhn[r] = (dh - (double)L.h[r] * dN) / Nr;
#pragma unroll
            for (int k = 0; k < N; ++k) dGn[r][k] = -(double)L.G[r][k] * (dN / Nr);
        }
        // rhs1 = -dGn' lam ; rhs2_s = dhn_A - dGn_A z
        double rhs1[N], rhs2[N];
#pragma unroll
        for (int k = 0; k < N; ++k) {
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < M; ++r) acc -= dGn[r][k] * L.qp.lam[r];
            rhs1[k] = acc;
        }
#pragma unroll
        for (int sl = 0; sl < N; ++sl) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < M; ++r) {
                if (r == aidx[sl]) {
                    double acc = dhn[r];
#pragma unroll
                    for (int k = 0; k < N; ++k) acc -= dGn[r][k] * L.qp.z[k];
                    v = acc;
                }
            }
            rhs2[sl] = (sl < nact) ? v : 0.0;
        }
        double dz[N];
        if (nact == N) {
            double A[N][N], b[N];
#pragma unroll
            for (int a = 0; a < N; ++a) {
                b[a] = rhs2[a];
#pragma unroll
                for (int k = 0; k < N; ++k) A[a][k] = GA[a][k];
            }
            gauss_solve<N>(A, b, dz);
        } else {
            // dlam = S^-1 (G_A P^-1 rhs1 - rhs2), dz = P^-1 (rhs1 - G_A' dlam)
            double PG[N][N], Pr1[N], S[N][N], w[N], dl[N];
#pragma unroll
            for (int k = 0; k < N; ++k) Pr1[k] = rhs1[k] / pd[k];
#pragma unroll
            for (int sl = 0; sl < N; ++sl)
#pragma unroll
                for (int k = 0; k < N; ++k) PG[sl][k] = GA[sl][k] / pd[k];
#pragma unroll
            for (int a = 0; a < N; ++a) {
#pragma unroll
                for (int b = 0; b < N; ++b) {
                    bool in = (a < nact) && (b < nact);
                    S[a][b] = in ? dotd<N>(GA[a], PG[b]) : (a == b ? 1.0 : 0.0);
                }
                w[a] = (a < nact) ? dotd<N>(GA[a], Pr1) - rhs2[a] : 0.0;
            }
            ldl_solve<N>(S, w, dl);
#pragma unroll
            for (int k = 0; k < N; ++k) {
                double acc = rhs1[k];
#pragma unroll
                for (int sl = 0; sl < N; ++sl) acc -= GA[sl][k] * ((sl < nact) ? dl[sl] : 0.0);
                dz[k] = acc / pd[k];
            }
        }
#pragma unroll
        for (int a = 0; a < NU; ++a) J[a][c] = (a == c ? 1.0 : 0.0) + dz[a];
    }
#pragma unroll
    for (int a = 0; a < NU; ++a) {
        float v = us[a] + (float)L.qp.z[a];
        bool pass = (v >= (float)prm.u_min[a]) && (v <= (float)prm.u_max[a]);  // torch.clamp backward
        double ga = pass ? (double)grad_u[i * NU + a] : 0.0;
#pragma unroll
        for (int c = 0; c < NU; ++c) J[a][c] *= ga;
    }
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        double acc = 0.0;
#pragma unroll
        for (int a = 0; a < NU; ++a) acc += J[a][c];
        grad_u_rl[i * NU + c] = (float)acc;
    }
}

template <int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_cascade(rcbf_params prm, int64_t B, const double* __restrict__ un,
                                                    const double* __restrict__ x, const double* __restrict__ mu,
                                                    const double* __restrict__ sigma, double* __restrict__ u_out,
                                                    int32_t* __restrict__ status_out, int32_t* fail_flag) {
    using D = Dims<MODE, K>;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    double xs[D::NS], us[D::NU], m[D::NS], s[D::NS];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        xs[k] = x[i * D::NS + k];
        m[k] = mu ? mu[i * D::NS + k] : 0.0;
        s[k] = sigma ? sigma[i * D::NS + k] : (double)prior_sigma<MODE>(k);
    }
#pragma unroll
    for (int c = 0; c < D::NU; ++c) us[c] = un[i * D::NU + c];
    double G[D::M][D::N], h[D::M], Nrm[D::M];
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS)
        cars_rows_cascade(prm, xs, us[0], G, h);
    else
        uni_rows_cascade<K>(prm, xs, us, m, s, G, h);
    normalize_rows<D::N, D::M, double>(G, h, Nrm, nullptr);
    double pd[D::N], q[D::N];
    cascade_P<MODE>(pd);
#pragma unroll
    for (int k = 0; k < D::N; ++k) q[k] = 0.0;
    PMat<D::N, true> pm;
    pmat_set_diag<D::N>(pm, pd);
    QPResult<D::N, D::M> res;
    qp_solve<D::N, D::M, true, double>(prm.solver, pm, q, G, h, prm.max_iter, prm.eps, res);
#pragma unroll
    for (int c = 0; c < D::NU; ++c) u_out[i * D::NU + c] = res.z[c];
    report(res.status, status_out, i, fail_flag);
}

// ---------------------------------------------------------------------------
// kernels: environments
// ---------------------------------------------------------------------------
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
    if constexpr ((kAblate & 8) != 0) {
#pragma unroll
        for (int k = 0; k < Dims<MODE, 1>::NO; ++k) o[k] = xs[k % Dims<MODE, 1>::NS];
    } else if constexpr (MODE == RCBF_MODE_SIMULATED_CARS)
        cars_obs(xs, o);
    else
        uni_obs(xs, o);
}

template <int MODE>
__global__ void __launch_bounds__(kBlock) k_env_reset(rcbf_params prm, int64_t B, const uint8_t* __restrict__ mask,
                                                      const double* __restrict__ noise, uint64_t seed,
                                                      int64_t off, double* __restrict__ x, double* __restrict__ aux,
                                                      int32_t* __restrict__ step, uint32_t* __restrict__ episode,
                                                      float* __restrict__ obs_out) {
    using D = Dims<MODE, 1>;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    if (mask && !mask[i]) return;
    double xs[D::NS], a;
    int st;
    uint32_t ep = episode ? episode[i] + 1u : 0u;
    env_reset_one<MODE>(noise, i, seed, off, ep, xs, a, st);
#pragma unroll
    for (int k = 0; k < D::NS; ++k) x[i * D::NS + k] = xs[k];
    aux[i] = a;
    step[i] = st;
    if (episode) episode[i] = ep;
    if (obs_out) {
        double o[D::NO];
        env_obs<MODE>(xs, o);
#pragma unroll
        for (int k = 0; k < D::NO; ++k) obs_out[i * D::NO + k] = (float)o[k];
    }
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
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    double xs[D::NS];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) xs[k] = x[i * D::NS + k];
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
#pragma unroll
    for (int k = 0; k < D::NS; ++k) x[i * D::NS + k] = xs[k];
    aux[i] = a;
    step[i] = st;
    double o[D::NO];
    env_obs<MODE>(xs, o);
#pragma unroll
    for (int k = 0; k < D::NO; ++k) {
        if (obs64) obs64[i * D::NO + k] = o[k];
        if (obs32) obs32[i * D::NO + k] = (float)o[k];
    }
}

// state32 = get_state(float(obs(x)))   (dynamics.py:190-232, via the fp32
// observation the policy sees: sac_cbf.py:61 then to_numpy/fp64/rescale/fp32)
template <int MODE>
__device__ __forceinline__ void state_from_env(const double* xs, float* s32, float* obs32) {
#pragma clang fp contract(off)
    double o[Dims<MODE, 1>::NO];
    env_obs<MODE>(xs, o);
#pragma unroll
    for (int k = 0; k < Dims<MODE, 1>::NO; ++k) obs32[k] = (float)o[k];
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
#pragma unroll
        for (int k = 0; k < 10; ++k) s32[k] = (float)((double)obs32[k] * ((k & 1) ? 30.0 : 100.0));
    } else {
        s32[0] = obs32[0];
        s32[1] = obs32[1];
        s32[2] = (float)atan2((double)obs32[3], (double)obs32[2]);
    }
}

// One fused safe step for one env; shared by k_safe_step and k_safe_rollout.
template <int MODE, int K>
__device__ __forceinline__ void safe_step_one(const rcbf_params& prm, int64_t i, double* xs, double& a, int& st,
                                              uint32_t& ep, const float* us, const float* m, const float* s,
                                              float* uf, float& rew, float& cst, bool& dn, bool& gm, int& status,
                                              int auto_reset, uint64_t seed, int64_t off) {
    using D = Dims<MODE, K>;
    float s32[D::NS], o32[D::NO];
    state_from_env<MODE>(xs, s32, o32);
    LayerState<MODE, K> L;
    layer_forward<MODE, K>(prm, s32, us, m, s, uf, L);
    status = L.qp.status;
    if constexpr ((kAblate & 4) != 0) {
#pragma unroll
        for (int k = 0; k < D::NS; ++k) xs[k] += 1e-3 * (double)uf[0];
        st += 1;
        rew = uf[0];
        cst = 0.0f;
        dn = st >= 300;
        gm = false;
    } else if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        CarsStepOut o;
        cars_env_step<float>(prm, xs, a, st, uf[0], o);
        rew = o.reward;
        cst = (float)o.cost;
        dn = o.done;
        gm = false;
    } else {
        UniStepOut o;
        uni_env_step<float>(prm, xs, a, st, uf, o);
        rew = (float)o.reward;
        cst = (float)o.cost;
        dn = o.done;
        gm = o.goal;
    }
    if (auto_reset && dn) {
        ep += 1u;
        env_reset_one<MODE>(nullptr, i, seed, off, ep, xs, a, st);
    }
}

template <int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_safe_step(rcbf_params prm, int64_t B, double* __restrict__ x,
                                                      double* __restrict__ aux, int32_t* __restrict__ step,
                                                      uint32_t* __restrict__ episode, const float* __restrict__ u_rl,
                                                      const float* __restrict__ mu, const float* __restrict__ sigma,
                                                      float* __restrict__ obs_out, float* __restrict__ u_out,
                                                      float* __restrict__ reward, float* __restrict__ cost,
                                                      uint8_t* __restrict__ done, uint8_t* __restrict__ goal_met,
                                                      int32_t* __restrict__ status_out, int32_t* fail_flag,
                                                      int auto_reset, uint64_t seed, int64_t off) {
    using D = Dims<MODE, K>;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    double xs[D::NS];
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        const double2* xv = reinterpret_cast<const double2*>(x + i * 10);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            double2 v = xv[k];
            xs[2 * k] = v.x;
            xs[2 * k + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < D::NS; ++k) xs[k] = x[i * D::NS + k];
    }
    double a = aux[i];
    int st = step[i];
    uint32_t ep = episode ? episode[i] : 0u;
    float us[D::NU], m[D::NS], s[D::NS], uf[D::NU];
#pragma unroll
    for (int c = 0; c < D::NU; ++c) us[c] = u_rl[i * D::NU + c];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        m[k] = mu ? mu[i * D::NS + k] : 0.0f;
        s[k] = sigma ? sigma[i * D::NS + k] : prior_sigma<MODE>(k);
    }
    float rew, cst;
    bool dn, gm;
    int status;
    const uint32_t ep0 = ep;
    safe_step_one<MODE, K>(prm, i, xs, a, st, ep, us, m, s, uf, rew, cst, dn, gm, status, auto_reset, seed, off);
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        double2* xv = reinterpret_cast<double2*>(x + i * 10);
#pragma unroll
        for (int k = 0; k < 5; ++k) xv[k] = make_double2(xs[2 * k], xs[2 * k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < D::NS; ++k) x[i * D::NS + k] = xs[k];
    }
    aux[i] = a;
    step[i] = st;
    if (episode && ep != ep0) episode[i] = ep;
    double o[D::NO];
    env_obs<MODE>(xs, o);
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS) {
        float2* ov = reinterpret_cast<float2*>(obs_out + i * 10);
#pragma unroll
        for (int k = 0; k < 5; ++k) ov[k] = make_float2((float)o[2 * k], (float)o[2 * k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < D::NO; ++k) obs_out[i * D::NO + k] = (float)o[k];
    }
#pragma unroll
    for (int c = 0; c < D::NU; ++c) u_out[i * D::NU + c] = uf[c];
    reward[i] = rew;
    cost[i] = cst;
    done[i] = dn;
    if (goal_met) goal_met[i] = gm;
    report(status, status_out, i, fail_flag);
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
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    double xs[D::NS];
#pragma unroll
    for (int k = 0; k < D::NS; ++k) xs[k] = x[i * D::NS + k];
    double a = aux[i];
    int st = step[i];
    uint32_t ep = episode ? episode[i] : 0u;
    const uint32_t ep0 = ep;
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
        safe_step_one<MODE, K>(prm, i, xs, a, st, ep, us, m, s, uf, rew, cst, dn, gm, status, 1, seed, off);
        rs += rew;
        cs += cst;
        nd += dn ? 1 : 0;
        worst = status > worst ? status : worst;
    }
#pragma unroll
    for (int k = 0; k < D::NS; ++k) x[i * D::NS + k] = xs[k];
    aux[i] = a;
    step[i] = st;
    if (episode && ep != ep0) episode[i] = ep;
    if (obs_out) {
        double o[D::NO];
        env_obs<MODE>(xs, o);
#pragma unroll
        for (int k = 0; k < D::NO; ++k) obs_out[i * D::NO + k] = (float)o[k];
    }
    reward_sum[i] = rs;
    cost_sum[i] = cs;
    n_done[i] = nd;
    if (worst != RCBF_QP_OK && fail_flag) atomicOr(fail_flag, 1 << worst);
}

// ---------------------------------------------------------------------------
// host dispatch helpers
// ---------------------------------------------------------------------------
int check_prm(const rcbf_params* prm) {
    if (!prm) return RCBF_E_NULL;
    if (prm->mode != RCBF_MODE_SIMULATED_CARS && prm->mode != RCBF_MODE_UNICYCLE) return RCBF_E_BAD_MODE;
    if (prm->mode == RCBF_MODE_UNICYCLE && (prm->num_hazards < 1 || prm->num_hazards > RCBF_MAX_HAZARDS))
        return RCBF_E_BAD_SHAPE;
    if (prm->solver != RCBF_SOLVER_ACTIVE_SET && prm->solver != RCBF_SOLVER_PDIPM) return RCBF_E_BAD_MODE;
    return 0;
}

inline int launch_status() { return (int)hipGetLastError(); }

// Dispatch F<MODE, K>(args...) over the unicycle hazard count.
#define RCBF_DISPATCH(prm, ...)                                                      \
    do {                                                                                \
        if ((prm)->mode == RCBF_MODE_SIMULATED_CARS) {                                  \
            constexpr int MODE_ = RCBF_MODE_SIMULATED_CARS;                             \
            constexpr int K_ = 1;                                                       \
            __VA_ARGS__;                                                                     \
        } else {                                                                        \
            constexpr int MODE_ = RCBF_MODE_UNICYCLE;                                   \
            switch ((prm)->num_hazards) {                                               \
                case 1: { constexpr int K_ = 1; __VA_ARGS__; } break;                        \
                case 2: { constexpr int K_ = 2; __VA_ARGS__; } break;                        \
                case 3: { constexpr int K_ = 3; __VA_ARGS__; } break;                        \
                case 4: { constexpr int K_ = 4; __VA_ARGS__; } break;                        \
                case 5: { constexpr int K_ = 5; __VA_ARGS__; } break;                        \
                case 6: { constexpr int K_ = 6; __VA_ARGS__; } break;                        \
                case 7: { constexpr int K_ = 7; __VA_ARGS__; } break;                        \
                default: { constexpr int K_ = 8; __VA_ARGS__; } break;                       \
            }                                                                           \
        }                                                                               \
    } while (0)

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

const char* rcbf_version(void) { return "rcbf_hip 0.1.0 (gfx950)"; }
int32_t rcbf_abi_version(void) { return RCBF_ABI_VERSION; }
int32_t rcbf_params_size(void) { return (int32_t)sizeof(rcbf_params); }

int rcbf_build(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl, const float* mu,
               const float* sigma, float* P_out, float* q_out, float* G_out, float* h_out, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_rl || !G_out || !h_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_build<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream, *prm,
                                           B, x, u_rl, mu, sigma, P_out, q_out, G_out, h_out));
    return launch_status();
}

int rcbf_build_f64(const rcbf_params* prm, int64_t B, const double* x, const double* u_nom, const double* mu,
                   const double* sigma, double* P_out, double* q_out, double* G_out, double* h_out,
                   hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_nom || !G_out || !h_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_build_f64<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream,
                                           *prm, B, x, u_nom, mu, sigma, P_out, q_out, G_out, h_out));
    return launch_status();
}

int rcbf_qp_solve(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P, const float* q,
                  const float* G, const float* h, int32_t normalize, float* z_out, double* lam_out,
                  int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    if (!prm) return RCBF_E_NULL;
    if (prm->solver != RCBF_SOLVER_ACTIVE_SET && prm->solver != RCBF_SOLVER_PDIPM) return RCBF_E_BAD_MODE;
    if (B < 0 || n < 1 || n > 3 || m < 1 || m > 16) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!P || !G || !h || !z_out) return RCBF_E_NULL;
    dim3 g(grid_for(B)), b(kBlock);
#define RCBF_QP_L(NN, MP) \
    hipLaunchKernelGGL((k_qp_solve<NN, MP>), g, b, 0, stream, *prm, B, m, P, q, G, h, normalize, z_out, lam_out, \
                       status_out, fail_flag)
#define RCBF_QP_M(NN)                  \
    do {                               \
        if (m <= 4)                    \
            RCBF_QP_L(NN, 4);          \
        else if (m <= 8)               \
            RCBF_QP_L(NN, 8);          \
        else if (m <= 12)              \
            RCBF_QP_L(NN, 12);         \
        else                           \
            RCBF_QP_L(NN, 16);         \
    } while (0)
    if (n == 1)
        RCBF_QP_M(1);
    else if (n == 2)
        RCBF_QP_M(2);
    else
        RCBF_QP_M(3);
#undef RCBF_QP_M
#undef RCBF_QP_L
    return launch_status();
}

int rcbf_safe_action(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl, const float* mu,
                     const float* sigma, float* u_out, int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_rl || !u_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_safe_action<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream,
                                           *prm, B, x, u_rl, mu, sigma, u_out, status_out, fail_flag));
    return launch_status();
}

int rcbf_safe_action_backward(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl,
                              const float* mu, const float* sigma, const float* grad_u, float* grad_u_rl,
                              hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_rl || !grad_u || !grad_u_rl) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_safe_action_bwd<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0,
                                           stream, *prm, B, x, u_rl, mu, sigma, grad_u, grad_u_rl));
    return launch_status();
}

int rcbf_cascade_u_safe(const rcbf_params* prm, int64_t B, const double* u_nom, const double* x, const double* mu,
                        const double* sigma, double* u_safe_out, int32_t* status_out, int32_t* fail_flag,
                        hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_nom || !u_safe_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_cascade<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream,
                                           *prm, B, u_nom, x, mu, sigma, u_safe_out, status_out, fail_flag));
    return launch_status();
}

int rcbf_env_reset(const rcbf_params* prm, int64_t B, const uint8_t* mask, const double* noise, uint64_t seed,
                   int64_t env_offset, double* x, double* aux, int32_t* step, uint32_t* episode, float* obs_out,
                   hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !aux || !step) return RCBF_E_NULL;
    if (prm->mode == RCBF_MODE_SIMULATED_CARS)
        hipLaunchKernelGGL((k_env_reset<RCBF_MODE_SIMULATED_CARS>), dim3(grid_for(B)), dim3(kBlock), 0, stream, *prm,
                           B, mask, noise, seed, env_offset, x, aux, step, episode, obs_out);
    else
        hipLaunchKernelGGL((k_env_reset<RCBF_MODE_UNICYCLE>), dim3(grid_for(B)), dim3(kBlock), 0, stream, *prm, B,
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
    dim3 g(grid_for(B)), b(kBlock);
    if (prm->mode == RCBF_MODE_SIMULATED_CARS) {
        if (action_f64)
            hipLaunchKernelGGL((k_env_step<RCBF_MODE_SIMULATED_CARS, double>), g, b, 0, stream, *prm, B, x, aux, step,
                               episode, (const double*)action, obs64_out, obs_out, reward, cost, done, goal_met,
                               auto_reset, seed, env_offset);
        else
            hipLaunchKernelGGL((k_env_step<RCBF_MODE_SIMULATED_CARS, float>), g, b, 0, stream, *prm, B, x, aux, step,
                               episode, (const float*)action, obs64_out, obs_out, reward, cost, done, goal_met,
                               auto_reset, seed, env_offset);
    } else {
        if (action_f64)
            hipLaunchKernelGGL((k_env_step<RCBF_MODE_UNICYCLE, double>), g, b, 0, stream, *prm, B, x, aux, step,
                               episode, (const double*)action, obs64_out, obs_out, reward, cost, done, goal_met,
                               auto_reset, seed, env_offset);
        else
            hipLaunchKernelGGL((k_env_step<RCBF_MODE_UNICYCLE, float>), g, b, 0, stream, *prm, B, x, aux, step,
                               episode, (const float*)action, obs64_out, obs_out, reward, cost, done, goal_met,
                               auto_reset, seed, env_offset);
    }
    return launch_status();
}

int rcbf_safe_step(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step, uint32_t* episode,
                   const float* u_rl, const float* mu, const float* sigma, float* obs_out, float* u_out,
                   float* reward, float* cost, uint8_t* done, uint8_t* goal_met, int32_t* status_out,
                   int32_t* fail_flag, int32_t auto_reset, uint64_t seed, int64_t env_offset, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !aux || !step || !u_rl || !obs_out || !u_out || !reward || !cost || !done) return RCBF_E_NULL;
    if (prm->mode == RCBF_MODE_SIMULATED_CARS && ((((uintptr_t)x) & 15) || (((uintptr_t)obs_out) & 7)))
        return RCBF_E_BAD_SHAPE;  // vectorised row access needs 16 B / 8 B alignment
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_safe_step<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream,
                                           *prm, B, x, aux, step, episode, u_rl, mu, sigma, obs_out, u_out, reward,
                                           cost, done, goal_met, status_out, fail_flag, auto_reset, seed, env_offset));
    return launch_status();
}

int rcbf_safe_rollout(const rcbf_params* prm, int64_t B, int32_t K, double* x, double* aux, int32_t* step,
                      uint32_t* episode, const float* u_rl, float* obs_out, float* reward_sum, float* cost_sum,
                      int32_t* n_done, int32_t* fail_flag, uint64_t seed, int64_t env_offset, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0 || K < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0 || K == 0) return 0;
    if (!x || !aux || !step || !u_rl || !reward_sum || !cost_sum || !n_done) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_safe_rollout<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream,
                                           *prm, B, K, x, aux, step, episode, u_rl, obs_out, reward_sum, cost_sum,
                                           n_done, fail_flag, seed, env_offset));
    return launch_status();
}

}  // extern "C"
