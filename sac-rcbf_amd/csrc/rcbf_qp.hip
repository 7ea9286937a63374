// rcbf_qp.hip -- generic QP and Cascade-layer kernels + C-ABI:
// rcbf_qp_solve (CBFQPLayer.solve_qp / cbf_layer), rcbf_cascade_u_safe
// (CascadeCBFLayer.get_u_safe).
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

// Generic QP (diff_cbf_qp.py:81-144): rows padded to MP with the never-active
// row (0 z <= 1); general SPD P (n <= 3).
template <int SOLVER, int N, int MP>
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
    qp_solve<SOLVER, N, MP, false, float>(pm, qd, Gl, hl, prm.max_iter, prm.eps, res);
#pragma unroll
    for (int k = 0; k < N; ++k) z_out[i * N + k] = (float)res.z[k];
    if (lam_out) {
#pragma unroll
        for (int r = 0; r < MP; ++r)
            if (r < m) lam_out[i * m + r] = res.lam[r];
    }
    report(res.status, status_out, i, fail_flag);
}

template <int SOLVER, int MODE, int K>
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
    normalize_rows<D::N, D::M, double>(G, h, Nrm, nullptr);  // cbf_qp.py:270-273
    double pd[D::N], q[D::N];
    cascade_P<MODE>(pd);
#pragma unroll
    for (int k = 0; k < D::N; ++k) q[k] = 0.0;
    PMat<D::N, true> pm;
    pmat_set_diag<D::N>(pm, pd);
    QPResult<D::N, D::M> res;
    if constexpr (MODE == RCBF_MODE_SIMULATED_CARS && SOLVER == RCBF_SOLVER_ACTIVE_SET)
        cars_qp_1d<double>(pm, G, h, res.z, res.status);
    else if constexpr (MODE == RCBF_MODE_UNICYCLE && SOLVER == RCBF_SOLVER_ACTIVE_SET)
        uni_qp_2d<K, double>(pm, G, h, res.z, res.status);
    else
        qp_solve<SOLVER, D::N, D::M, true, double>(pm, q, G, h, prm.max_iter, prm.eps, res);
#pragma unroll
    for (int c = 0; c < D::NU; ++c) u_out[i * D::NU + c] = res.z[c];
    report(res.status, status_out, i, fail_flag);
}

}  // namespace

extern "C" {

int rcbf_qp_solve(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P, const float* q,
                  const float* G, const float* h, int32_t normalize, float* z_out, double* lam_out,
                  int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    if (!prm) return RCBF_E_NULL;
    if (prm->solver != RCBF_SOLVER_ACTIVE_SET && prm->solver != RCBF_SOLVER_PDIPM && prm->solver != RCBF_SOLVER_GI)
        return RCBF_E_BAD_MODE;
    if (B < 0 || n < 1 || n > 3 || m < 1 || m > 16) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!P || !G || !h || !z_out) return RCBF_E_NULL;
    dim3 g(grid_for(B)), b(kBlock);
#define RCBF_QP_L(NN, MP)                                                                                         \
    do {                                                                                                          \
        if (prm->solver == RCBF_SOLVER_PDIPM)                                                                     \
            hipLaunchKernelGGL((k_qp_solve<RCBF_SOLVER_PDIPM, NN, MP>), g, b, 0, stream, *prm, B, m, P, q, G, h, \
                               normalize, z_out, lam_out, status_out, fail_flag);                                 \
        else                                                                                                      \
            hipLaunchKernelGGL((k_qp_solve<RCBF_SOLVER_GI, NN, MP>), g, b, 0, stream, *prm, B, m, P, q, G, h,    \
                               normalize, z_out, lam_out, status_out, fail_flag);                                 \
    } while (0)
#define RCBF_QP_M(NN)           \
    do {                        \
        if (m <= 4)             \
            RCBF_QP_L(NN, 4);   \
        else if (m <= 8)        \
            RCBF_QP_L(NN, 8);   \
        else if (m <= 12)       \
            RCBF_QP_L(NN, 12);  \
        else                    \
            RCBF_QP_L(NN, 16);  \
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

int rcbf_cascade_u_safe(const rcbf_params* prm, int64_t B, const double* u_nom, const double* x, const double* mu,
                        const double* sigma, double* u_safe_out, int32_t* status_out, int32_t* fail_flag,
                        hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_nom || !u_safe_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_cascade<SOLVER_, MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream,
                                          *prm, B, u_nom, x, mu, sigma, u_safe_out, status_out, fail_flag));
    return launch_status();
}

}  // extern "C"
