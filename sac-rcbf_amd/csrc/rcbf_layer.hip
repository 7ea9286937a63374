// rcbf_layer.hip -- CBFQPLayer kernels + C-ABI (include/rcbf_hip.h):
// rcbf_build, rcbf_build_f64, rcbf_safe_action, rcbf_safe_action_backward.
// One env per lane; the env's rows, QP iterate and active set stay in VGPRs.
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

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

// FROM_OBS: x is the (B, n_o) observation and the state comes from
// DynamicsModel.get_state in-kernel (RCBF_SAC.get_safe_action, sac_cbf.py:218-238).
template <int MODE, int K, bool FROM_OBS = false>
__device__ __forceinline__ void load_layer_inputs(int64_t i, const float* x, const float* u, const float* mu,
                                                  const float* sigma, float* xs, float* us, float* m, float* s) {
    using D = Dims<MODE, K>;
    if constexpr (FROM_OBS) {
        constexpr int NO = Dims<MODE, 1>::NO;
        float o[NO];
#pragma unroll
        for (int k = 0; k < NO; ++k) o[k] = x[i * NO + k];
        state_from_obs32<MODE>(o, xs);
    }
#pragma unroll
    for (int k = 0; k < D::NS; ++k) {
        if constexpr (!FROM_OBS) xs[k] = x[i * D::NS + k];
        m[k] = mu ? mu[i * D::NS + k] : 0.0f;
        s[k] = sigma ? sigma[i * D::NS + k] : prior_sigma<MODE>(k);
    }
#pragma unroll
    for (int c = 0; c < D::NU; ++c) us[c] = u[i * D::NU + c];
}

template <int SOLVER, int MODE, int K, bool FROM_OBS = false, int BS = kBlock>
__global__ void __launch_bounds__(BS) k_safe_action(rcbf_params prm, int64_t B, const float* __restrict__ x,
                                                        const float* __restrict__ u, const float* __restrict__ mu,
                                                        const float* __restrict__ sigma, float* __restrict__ u_out,
                                                        int32_t* __restrict__ status_out, int32_t* fail_flag) {
    using D = Dims<MODE, K>;
    int64_t i = env_index<BS>();
    if (i >= B) return;
    float xs[D::NS], us[D::NU], m[D::NS], s[D::NS], uf[D::NU];
    load_layer_inputs<MODE, K, FROM_OBS>(i, x, u, mu, sigma, xs, us, m, s);
    LayerState<MODE, K> L;
    layer_forward<SOLVER, MODE, K>(prm, xs, us, m, s, uf, L);
#pragma unroll
    for (int c = 0; c < D::NU; ++c) u_out[i * D::NU + c] = uf[c];
    report(L.qp.status, status_out, i, fail_flag);
}

// Multipliers of the layer's QP at its closed-form optimum (diagonal P,
// q = 0, the normalised rows in L): the rows with G_r z = h_r (to 1e-9
// relative) form A, and lam_A solves P z + G_A' lam_A = 0 on them.  Returns
// false for a degenerate point (more than n rows tight, a negative multiplier
// or a stationarity residual); the caller then runs Goldfarb-Idnani.
template <int MODE, int K>
__device__ __forceinline__ bool layer_multipliers(const double* pd, LayerState<MODE, K>& L) {
    using D = Dims<MODE, K>;
    constexpr int N = D::N, M = D::M;
    double GA[N][N], ip[N];
#pragma unroll
    for (int k = 0; k < N; ++k) ip[k] = 1.0 / pd[k];
    int nact = 0, aidx[N];
    uint32_t amask = 0;
    bool ok = true;
#pragma unroll
    for (int sl = 0; sl < N; ++sl) {
        aidx[sl] = -1;
#pragma unroll
        for (int k = 0; k < N; ++k) GA[sl][k] = 0.0;
    }
#pragma unroll
    for (int r = 0; r < M; ++r) {
        double v = -(double)L.h[r];
#pragma unroll
        for (int k = 0; k < N; ++k) v = fma((double)L.G[r][k], L.qp.z[k], v);
        const bool tight = fabs(v) <= 1e-9 * (1.0 + fabs((double)L.h[r]));
        ok = ok && !(tight && nact >= N);
        const bool a = tight && nact < N;
#pragma unroll
        for (int sl = 0; sl < N; ++sl) {
            const bool here = a && (sl == nact);
#pragma unroll
            for (int k = 0; k < N; ++k) GA[sl][k] = here ? (double)L.G[r][k] : GA[sl][k];
            aidx[sl] = here ? r : aidx[sl];
        }
        amask |= a ? (1u << r) : 0u;
        nact += a ? 1 : 0;
    }
    double S[N][N], w[N], lam[N];
#pragma unroll
    for (int a = 0; a < N; ++a) {
#pragma unroll
        for (int b = 0; b < N; ++b) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < N; ++k) acc = fma(GA[a][k] * ip[k], GA[b][k], acc);
            S[a][b] = (a < nact && b < nact) ? acc : (a == b ? 1.0 : 0.0);
        }
        w[a] = (a < nact) ? -dotd<N>(GA[a], L.qp.z) : 0.0;
    }
    ok = ok && ldl_solve<N>(S, w, lam);
    double scale = 1.0;
#pragma unroll
    for (int sl = 0; sl < N; ++sl) scale = fmax(scale, fabs(lam[sl]));
#pragma unroll
    for (int sl = 0; sl < N; ++sl) ok = ok && (sl >= nact || lam[sl] >= -1e-9 * scale);
#pragma unroll
    for (int k = 0; k < N; ++k) {  // stationarity: P z + G_A' lam = 0
        double acc = pd[k] * L.qp.z[k];
#pragma unroll
        for (int sl = 0; sl < N; ++sl) acc = fma((sl < nact) ? GA[sl][k] : 0.0, lam[sl], acc);
        ok = ok && fabs(acc) <= 1e-7 * scale * (1.0 + fabs(pd[k] * L.qp.z[k]));
    }
#pragma unroll
    for (int r = 0; r < M; ++r) {
        double l = 0.0;
#pragma unroll
        for (int sl = 0; sl < N; ++sl) l = (sl < nact && aidx[sl] == r) ? fmax(lam[sl], 0.0) : l;
        L.qp.lam[r] = l;
    }
    L.qp.active = amask;
    L.qp.nact = nact;
    return ok;
}

// The forward with multipliers for the backward.  The exact solver (the
// default): the closed-form optimum on the normalised rows -- the very z the
// forward returns -- with its multipliers from stationarity; a lane whose
// point is degenerate re-solves with Goldfarb-Idnani (the rows are the same,
// so it finds the same optimum).  Other solvers: their own multipliers.
template <int SOLVER, int MODE, int K>
__device__ __forceinline__ void layer_forward_lam(const rcbf_params& prm, const float* xs, const float* us,
                                                  const float* m, const float* s, float* uf,
                                                  LayerState<MODE, K>& L) {
    using D = Dims<MODE, K>;
    if constexpr (SOLVER == RCBF_SOLVER_ACTIVE_SET) {
        layer_forward<SOLVER, MODE, K>(prm, xs, us, m, s, uf, L);  // normalised rows, closed form
        double pd[D::N];
        diff_P<MODE>(pd);
        if (!layer_multipliers<MODE, K>(pd, L)) {
            PMat<D::N, true> pm;
            double q[D::N];
#pragma unroll
            for (int k = 0; k < D::N; ++k) q[k] = 0.0;
            pmat_set_diag<D::N>(pm, pd);
            qp_solve<SOLVER, D::N, D::M, true, float>(pm, q, L.G, L.h, prm.max_iter, prm.eps, L.qp);
        }
    } else {
        layer_forward<SOLVER, MODE, K, true>(prm, xs, us, m, s, uf, L);
    }
}

// d(final)/d(u_rl) on the active set of the exact optimum: the implicit-KKT
// derivative qpth's QPFunction.backward approximates (D = lam/s over all
// rows), through the row normaliser (torch.max routes dN to its argmax, the h
// entry or a G entry that does not depend on u) and the clamp (torch.clamp
// backward passes where lo <= v <= hi).  dh_r/du_c is closed form:
//   CBF rows: dh/du = Lg (cars) or a_j (unicycle) = -G_raw[r][c];
//   actuator rows (u_max - u, -u_min + u): -1 / +1.
// J[a][c] = d(u_a + z_a) / d u_c; pass[a]: the clamp passes action a's gradient;
// uf / status: the forward's output (the plain forward's, bit for bit).
template <int SOLVER, int MODE, int K>
__device__ __forceinline__ void layer_jacobian(const rcbf_params& prm, const float* xs, const float* us,
                                               const float* m, const float* s,
                                               double (&J)[Dims<MODE, K>::NU][Dims<MODE, K>::NU],
                                               bool (&pass)[Dims<MODE, K>::NU], float* uf, int& status) {
    using D = Dims<MODE, K>;
    constexpr int N = D::N, M = D::M, NU = D::NU;
    LayerState<MODE, K> L;
    layer_forward_lam<SOLVER, MODE, K>(prm, xs, us, m, s, uf, L);
    status = L.qp.status;
    double pd[N];
    diff_P<MODE>(pd);
    // active rows (slots) of the solution
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
        bool a = ((L.qp.active >> r) & 1u) && (nact < N);
#pragma unroll
        for (int sl = 0; sl < N; ++sl) {
            bool here = a && (sl == nact);
#pragma unroll
            for (int k = 0; k < N; ++k) GA[sl][k] = here ? (double)L.G[r][k] : GA[sl][k];
            aidx[sl] = here ? r : aidx[sl];
        }
        nact += a ? 1 : 0;
    }
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        double dGn[M][N], dhn[M];
#pragma unroll
        for (int r = 0; r < M; ++r) {
            double dh;
            constexpr int K0 = M - 2 * NU;  // first actuator row
            if (r < K0) {
                dh = -(double)L.Graw[r][c];
            } else {
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
        // P dz + dGn' lam + G_A' dlam = 0 ;  G_A dz = dhn_A - dGn_A z
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
        if (nact == N) {  // vertex: dz = G_A^-1 rhs2
            double A[N][N], b[N];
#pragma unroll
            for (int a = 0; a < N; ++a) {
                b[a] = rhs2[a];
#pragma unroll
                for (int k = 0; k < N; ++k) A[a][k] = GA[a][k];
            }
            gauss_solve<N>(A, b, dz);
        } else {  // dlam = S^-1 (G_A P^-1 rhs1 - rhs2), dz = P^-1 (rhs1 - G_A' dlam)
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
        pass[a] = (v >= (float)prm.u_min[a]) && (v <= (float)prm.u_max[a]);
    }
}

// the backward, recomputing the forward: grad_u_rl_c = sum over the passing a of grad_u_a J[a][c]
template <int SOLVER, int MODE, int K, bool FROM_OBS = false, int BS = kBlock>
__global__ void __launch_bounds__(BS) k_safe_action_bwd(rcbf_params prm, int64_t B, const float* __restrict__ x,
                                                        const float* __restrict__ u, const float* __restrict__ mu,
                                                        const float* __restrict__ sigma,
                                                        const float* __restrict__ grad_u,
                                                        float* __restrict__ grad_u_rl) {
    using D = Dims<MODE, K>;
    constexpr int NU = D::NU;
    int64_t i = env_index<BS>();
    if (i >= B) return;
    float xs[D::NS], us[NU], m[D::NS], s[D::NS];
    load_layer_inputs<MODE, K, FROM_OBS>(i, x, u, mu, sigma, xs, us, m, s);
    double J[NU][NU];
    bool pass[NU];
    float uf[NU];
    int status;
    layer_jacobian<SOLVER, MODE, K>(prm, xs, us, m, s, J, pass, uf, status);
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        double acc = 0.0;
#pragma unroll
        for (int a = 0; a < NU; ++a) acc += pass[a] ? (double)grad_u[i * NU + a] * J[a][c] : 0.0;
        grad_u_rl[i * NU + c] = (float)acc;
    }
}

// The forward that also keeps what its backward needs (like qpth's
// QPFunction keeping zhats): u_out exactly as k_safe_action, plus the
// Jacobian (B, n_u, n_u) f64 with the clamp folded in (a saturated action's
// row holds the marker RCBF_JAC_NO_GRAD, a NaN with its own payload: "no
// gradient"), so the backward is one small elementwise launch (k_apply_jac)
// instead of a second solve; it computes what k_safe_action_bwd computes, bit
// for bit.  Only the marker's exact bit pattern means "no gradient": a NaN
// that the solve itself produces (a degenerate active set) has another
// pattern and propagates into the gradient as it does in k_safe_action_bwd.
template <int SOLVER, int MODE, int K, bool FROM_OBS = false, int BS = kBlock>
__global__ void __launch_bounds__(BS) k_safe_action_jac(rcbf_params prm, int64_t B, const float* __restrict__ x,
                                                        const float* __restrict__ u, const float* __restrict__ mu,
                                                        const float* __restrict__ sigma, float* __restrict__ u_out,
                                                        double* __restrict__ jac, int32_t* __restrict__ status_out,
                                                        int32_t* fail_flag) {
    using D = Dims<MODE, K>;
    constexpr int NU = D::NU;
    int64_t i = env_index<BS>();
    if (i >= B) return;
    float xs[D::NS], us[NU], m[D::NS], s[D::NS], uf[NU];
    load_layer_inputs<MODE, K, FROM_OBS>(i, x, u, mu, sigma, xs, us, m, s);
    double J[NU][NU];
    bool pass[NU];
    int status;
    layer_jacobian<SOLVER, MODE, K>(prm, xs, us, m, s, J, pass, uf, status);
#pragma unroll
    for (int c = 0; c < NU; ++c) u_out[i * NU + c] = uf[c];
    report(status, status_out, i, fail_flag);
#pragma unroll
    for (int a = 0; a < NU; ++a)
#pragma unroll
        for (int c = 0; c < NU; ++c)
            jac[(i * NU + a) * NU + c] = pass[a] ? J[a][c] : __longlong_as_double((long long)RCBF_JAC_NO_GRAD);
}

template <int NU, int BS>
__global__ void __launch_bounds__(BS) k_apply_jac(int64_t B, const double* __restrict__ jac,
                                                  const float* __restrict__ grad_u, float* __restrict__ grad_u_rl) {
    int64_t i = env_index<BS>();
    if (i >= B) return;
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        double acc = 0.0;
#pragma unroll
        for (int a = 0; a < NU; ++a) {
            const double j = jac[(i * NU + a) * NU + c];
            const bool no_grad = (unsigned long long)__double_as_longlong(j) == RCBF_JAC_NO_GRAD;
            acc += no_grad ? 0.0 : (double)grad_u[i * NU + a] * j;
        }
        grad_u_rl[i * NU + c] = (float)acc;
    }
}

}  // namespace

extern "C" {

int rcbf_build(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl, const float* mu,
               const float* sigma, float* P_out, float* q_out, float* G_out, float* h_out, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_rl || !G_out || !h_out) return RCBF_E_NULL;
    RCBF_DISPATCH_MODE(prm, hipLaunchKernelGGL((k_build<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream,
                                               *prm, B, x, u_rl, mu, sigma, P_out, q_out, G_out, h_out));
    return launch_status();
}

int rcbf_build_f64(const rcbf_params* prm, int64_t B, const double* x, const double* u_nom, const double* mu,
                   const double* sigma, double* P_out, double* q_out, double* G_out, double* h_out,
                   hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_nom || !G_out || !h_out) return RCBF_E_NULL;
    RCBF_DISPATCH_MODE(prm, hipLaunchKernelGGL((k_build_f64<MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0,
                                               stream, *prm, B, x, u_nom, mu, sigma, P_out, q_out, G_out, h_out));
    return launch_status();
}

int rcbf_safe_action(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl, const float* mu,
                     const float* sigma, float* u_out, int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_rl || !u_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, RCBF_BS_LAUNCH_S(SOLVER_, B, (k_safe_action<SOLVER_, MODE_, K_, false, BS_>), stream, *prm, B, x, u_rl, mu,
                                      sigma, u_out, status_out, fail_flag));
    return launch_status();
}

int rcbf_safe_action_backward(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl,
                              const float* mu, const float* sigma, const float* grad_u, float* grad_u_rl,
                              hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_rl || !grad_u || !grad_u_rl) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, RCBF_BS_LAUNCH_S(SOLVER_, B, (k_safe_action_bwd<SOLVER_, MODE_, K_, false, BS_>), stream, *prm, B, x, u_rl,
                                      mu, sigma, grad_u, grad_u_rl));
    return launch_status();
}

int rcbf_obs_safe_action(const rcbf_params* prm, int64_t B, const float* obs, const float* u_rl, const float* mu,
                         const float* sigma, float* u_out, int32_t* status_out, int32_t* fail_flag,
                         hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!obs || !u_rl || !u_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, RCBF_BS_LAUNCH_S(SOLVER_, B, (k_safe_action<SOLVER_, MODE_, K_, true, BS_>), stream, *prm, B, obs, u_rl, mu,
                                      sigma, u_out, status_out, fail_flag));
    return launch_status();
}

int rcbf_obs_safe_action_backward(const rcbf_params* prm, int64_t B, const float* obs, const float* u_rl,
                                  const float* mu, const float* sigma, const float* grad_u, float* grad_u_rl,
                                  hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!obs || !u_rl || !grad_u || !grad_u_rl) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, RCBF_BS_LAUNCH_S(SOLVER_, B, (k_safe_action_bwd<SOLVER_, MODE_, K_, true, BS_>), stream, *prm, B, obs,
                                      u_rl, mu, sigma, grad_u, grad_u_rl));
    return launch_status();
}

int rcbf_safe_action_jac(const rcbf_params* prm, int64_t B, const float* x, const float* u_rl, const float* mu,
                         const float* sigma, float* u_out, double* jac_out, int32_t* status_out, int32_t* fail_flag,
                         hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_rl || !u_out || !jac_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, RCBF_BS_LAUNCH_S(SOLVER_, B, (k_safe_action_jac<SOLVER_, MODE_, K_, false, BS_>), stream, *prm, B, x, u_rl,
                                      mu, sigma, u_out, jac_out, status_out, fail_flag));
    return launch_status();
}

int rcbf_obs_safe_action_jac(const rcbf_params* prm, int64_t B, const float* obs, const float* u_rl,
                             const float* mu, const float* sigma, float* u_out, double* jac_out,
                             int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!obs || !u_rl || !u_out || !jac_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, RCBF_BS_LAUNCH_S(SOLVER_, B, (k_safe_action_jac<SOLVER_, MODE_, K_, true, BS_>), stream, *prm, B, obs,
                                      u_rl, mu, sigma, u_out, jac_out, status_out, fail_flag));
    return launch_status();
}

int rcbf_safe_action_apply_jac(int64_t B, int32_t n_u, const double* jac, const float* grad_u, float* grad_u_rl,
                               hipStream_t stream) {
    if (B < 0 || (n_u != 1 && n_u != 2)) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!jac || !grad_u || !grad_u_rl) return RCBF_E_NULL;
    if (n_u == 1)
        RCBF_BS_LAUNCH(B, (k_apply_jac<1, BS_>), stream, B, jac, grad_u, grad_u_rl);
    else
        RCBF_BS_LAUNCH(B, (k_apply_jac<2, BS_>), stream, B, jac, grad_u, grad_u_rl);
    return launch_status();
}

}  // extern "C"
