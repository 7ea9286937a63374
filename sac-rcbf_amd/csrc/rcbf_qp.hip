// rcbf_qp.hip -- generic QP and Cascade-layer kernels + C-ABI:
// rcbf_qp_solve / rcbf_qp_backward (CBFQPLayer.solve_qp / cbf_layer and their
// autograd), rcbf_qp_solve_f64 (CascadeCBFLayer.solve_qp),
// rcbf_cascade_u_safe (CascadeCBFLayer.get_u_safe).
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

// Generic QP (diff_cbf_qp.py:81-144; fp64 inputs: CascadeCBFLayer.solve_qp,
// cbf_qp.py:242-286): rows padded to MP with the never-active row
// (0 z <= 1); general SPD P (n <= 3).  T = float: the fp32 rows of the diff
// layer (z returned as fp32, the reference's .float()); T = double: fp64
// throughout.
template <int SOLVER, int N, int MP, typename T>
__global__ void __launch_bounds__(kBlock) k_qp_solve(rcbf_params prm, int64_t B, int m, const T* __restrict__ P,
                                                     const T* __restrict__ q, const T* __restrict__ G,
                                                     const T* __restrict__ h, int normalize,
                                                     T* __restrict__ z_out, double* __restrict__ lam_out,
                                                     int32_t* __restrict__ status_out, int32_t* fail_flag) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    T Gl[MP][N], hl[MP], Nrm[MP];
#pragma unroll
    for (int r = 0; r < MP; ++r) {
        bool in = r < m;
#pragma unroll
        for (int k = 0; k < N; ++k) Gl[r][k] = in ? G[(i * m + r) * N + k] : T(0);
        hl[r] = in ? h[i * m + r] : T(1);
    }
    if (normalize) normalize_rows<N, MP, T>(Gl, hl, Nrm, nullptr);
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
    qp_solve<SOLVER, N, MP, false, T>(pm, qd, Gl, hl, prm.max_iter, prm.eps, res);
#pragma unroll
    for (int k = 0; k < N; ++k) z_out[i * N + k] = (T)res.z[k];
    if (lam_out) {
#pragma unroll
        for (int r = 0; r < MP; ++r)
            if (r < m) lam_out[i * m + r] = res.lam[r];
    }
    report(res.status, status_out, i, fail_flag);
}

// Backward of k_qp_solve: CBFQPLayer.cbf_layer / solve_qp under autograd
// (diff_cbf_qp.py:81-144; the reference differentiates through qpth's
// QPFunction.backward, OptNet eq. 7-8, and through the row normaliser with
// torch autograd).  The forward is recomputed in-kernel with the exact
// Goldfarb-Idnani solver (z, multipliers lam, active set A), then the adjoint
// KKT system on A
//     P dz + G_A' eta = -grad_z,    G_A dz = 0
// gives (eta = D(lam) d_lam of OptNet; inactive rows carry eta = 0)
//     grad_q = dz,  grad_P = (dz z' + z dz') / 2,
//     grad_Gn = eta z' + lam dz',  grad_hn = -eta.
// With normalize, grad_Gn / grad_hn are pulled back through
// Gn = G / N, hn = h / N, N = max(|G_r|, |h_r|) (torch.max routes dN to the
// first maximal entry, d|x|/dx = sgn x).  Every output is [nullable].
template <int N, int MP>
__global__ void __launch_bounds__(kBlock) k_qp_bwd(rcbf_params prm, int64_t B, int m, const float* __restrict__ P,
                                                   const float* __restrict__ q, const float* __restrict__ G,
                                                   const float* __restrict__ h, int normalize,
                                                   const float* __restrict__ grad_z, float* __restrict__ gP,
                                                   float* __restrict__ gq, float* __restrict__ gG,
                                                   float* __restrict__ gh) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    float Gl[MP][N], hl[MP], Nrm[MP];
    int amax[MP];
#pragma unroll
    for (int r = 0; r < MP; ++r) {
        bool in = r < m;
#pragma unroll
        for (int k = 0; k < N; ++k) Gl[r][k] = in ? G[(i * m + r) * N + k] : 0.0f;
        hl[r] = in ? h[i * m + r] : 1.0f;
        float mx = fabsf(Gl[r][0]);
        int a = 0;
#pragma unroll
        for (int k = 1; k < N; ++k) {
            bool gt = fabsf(Gl[r][k]) > mx;
            a = gt ? k : a;
            mx = gt ? fabsf(Gl[r][k]) : mx;
        }
        amax[r] = (fabsf(hl[r]) > mx) ? N : a;
        Nrm[r] = 1.0f;
    }
    if (normalize) normalize_rows<N, MP, float>(Gl, hl, Nrm, nullptr);
    double Pin[N][N], qd[N], g[N];
#pragma unroll
    for (int a = 0; a < N; ++a) {
        qd[a] = q ? (double)q[i * N + a] : 0.0;
        g[a] = (double)grad_z[i * N + a];
#pragma unroll
        for (int b = 0; b < N; ++b) Pin[a][b] = (double)P[(i * N + a) * N + b];
    }
    PMat<N, false> pm;
    pmat_set_full<N>(pm, Pin);
    QPResult<N, MP> res;
    gi_solve<N, MP, false, float>(pm, qd, Gl, hl, 4 * (MP + N) + 8, res);
    // active rows in slots
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
    for (int r = 0; r < MP; ++r) {
        bool a = ((res.active >> r) & 1u) && (nact < N);
#pragma unroll
        for (int sl = 0; sl < N; ++sl) {
            bool here = a && (sl == nact);
#pragma unroll
            for (int k = 0; k < N; ++k) GA[sl][k] = here ? (double)Gl[r][k] : GA[sl][k];
            aidx[sl] = here ? r : aidx[sl];
        }
        nact += a ? 1 : 0;
    }
    double dz[N], eta[N];
    if (nact == N) {  // vertex: dz = 0, G_A' eta = -g
        double A[N][N], b[N];
#pragma unroll
        for (int a = 0; a < N; ++a) {
            b[a] = -g[a];
            dz[a] = 0.0;
#pragma unroll
            for (int k = 0; k < N; ++k) A[a][k] = GA[k][a];
        }
        gauss_solve<N>(A, b, eta);
    } else {  // (G_A P^-1 G_A') eta = -G_A P^-1 g,  dz = -P^-1 (g + G_A' eta)
        double Pg[N], PG[N][N], S[N][N], w[N], t[N];
        pm.inv_apply(g, Pg);
#pragma unroll
        for (int sl = 0; sl < N; ++sl) pm.inv_apply(GA[sl], PG[sl]);
#pragma unroll
        for (int a = 0; a < N; ++a) {
#pragma unroll
            for (int b = 0; b < N; ++b) {
                bool in = (a < nact) && (b < nact);
                S[a][b] = in ? dotd<N>(GA[a], PG[b]) : (a == b ? 1.0 : 0.0);
            }
            w[a] = (a < nact) ? -dotd<N>(GA[a], Pg) : 0.0;
        }
        ldl_solve<N>(S, w, eta);
#pragma unroll
        for (int k = 0; k < N; ++k) {
            double acc = g[k];
#pragma unroll
            for (int sl = 0; sl < N; ++sl) acc += (sl < nact) ? GA[sl][k] * eta[sl] : 0.0;
            t[k] = acc;
        }
        pm.inv_apply(t, dz);
#pragma unroll
        for (int k = 0; k < N; ++k) dz[k] = -dz[k];
    }
    const double* z = res.z;
    if (gq) {
#pragma unroll
        for (int a = 0; a < N; ++a) gq[i * N + a] = (float)dz[a];
    }
    if (gP) {
#pragma unroll
        for (int a = 0; a < N; ++a)
#pragma unroll
            for (int b = 0; b < N; ++b) gP[(i * N + a) * N + b] = (float)(0.5 * (dz[a] * z[b] + z[a] * dz[b]));
    }
    if (gG || gh) {
#pragma unroll
        for (int r = 0; r < MP; ++r) {
            if (r >= m) continue;
            double er = 0.0;
#pragma unroll
            for (int sl = 0; sl < N; ++sl) er = (aidx[sl] == r) ? eta[sl] : er;
            double gGn[N], ghn = -er;
#pragma unroll
            for (int k = 0; k < N; ++k) gGn[k] = er * z[k] + res.lam[r] * dz[k];
            double dN = 0.0, nr = 1.0;
            if (normalize) {
                nr = (double)Nrm[r];
                double acc = ghn * (double)hl[r];
#pragma unroll
                for (int k = 0; k < N; ++k) acc += gGn[k] * (double)Gl[r][k];
                dN = -acc / nr;
            }
            auto sgn = [](float v) { return v > 0.0f ? 1.0 : (v < 0.0f ? -1.0 : 0.0); };
            if (gG) {
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    double v = gGn[k] / nr + ((normalize && amax[r] == k) ? dN * sgn(Gl[r][k]) : 0.0);
                    gG[(i * m + r) * N + k] = (float)v;
                }
            }
            if (gh) gh[i * m + r] = (float)(ghn / nr + ((normalize && amax[r] == N) ? dN * sgn(hl[r]) : 0.0));
        }
    }
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

template <typename T>
int qp_solve_launch(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const T* P, const T* q, const T* G,
                    const T* h, int32_t normalize, T* z_out, double* lam_out, int32_t* status_out,
                    int32_t* fail_flag, hipStream_t stream) {
    if (!prm) return RCBF_E_NULL;
    if (prm->solver != RCBF_SOLVER_ACTIVE_SET && prm->solver != RCBF_SOLVER_PDIPM && prm->solver != RCBF_SOLVER_GI)
        return RCBF_E_BAD_MODE;
    if (B < 0 || n < 1 || n > 3 || m < 1 || m > 16) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!P || !G || !h || !z_out) return RCBF_E_NULL;
    dim3 g(grid_for(B)), b(kBlock);
#define RCBF_QP_L(NN, MP)                                                                                      \
    do {                                                                                                       \
        if (prm->solver == RCBF_SOLVER_PDIPM)                                                                  \
            hipLaunchKernelGGL((k_qp_solve<RCBF_SOLVER_PDIPM, NN, MP, T>), g, b, 0, stream, *prm, B, m, P, q, \
                               G, h, normalize, z_out, lam_out, status_out, fail_flag);                        \
        else                                                                                                   \
            hipLaunchKernelGGL((k_qp_solve<RCBF_SOLVER_GI, NN, MP, T>), g, b, 0, stream, *prm, B, m, P, q, G, \
                               h, normalize, z_out, lam_out, status_out, fail_flag);                           \
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

}  // namespace

extern "C" {

int rcbf_qp_solve(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P, const float* q,
                  const float* G, const float* h, int32_t normalize, float* z_out, double* lam_out,
                  int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    return qp_solve_launch<float>(prm, B, n, m, P, q, G, h, normalize, z_out, lam_out, status_out, fail_flag, stream);
}

int rcbf_qp_solve_f64(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const double* P, const double* q,
                      const double* G, const double* h, int32_t normalize, double* z_out, double* lam_out,
                      int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    return qp_solve_launch<double>(prm, B, n, m, P, q, G, h, normalize, z_out, lam_out, status_out, fail_flag,
                                   stream);
}

int rcbf_qp_backward(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P, const float* q,
                     const float* G, const float* h, int32_t normalize, const float* grad_z, float* grad_P,
                     float* grad_q, float* grad_G, float* grad_h, hipStream_t stream) {
    if (!prm) return RCBF_E_NULL;
    if (B < 0 || n < 1 || n > 3 || m < 1 || m > 16) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!P || !G || !h || !grad_z) return RCBF_E_NULL;
    dim3 g(grid_for(B)), b(kBlock);
#define RCBF_QPB_L(NN, MP)                                                                                     \
    hipLaunchKernelGGL((k_qp_bwd<NN, MP>), g, b, 0, stream, *prm, B, m, P, q, G, h, normalize, grad_z, grad_P, \
                       grad_q, grad_G, grad_h)
#define RCBF_QPB_M(NN)           \
    do {                         \
        if (m <= 4)              \
            RCBF_QPB_L(NN, 4);   \
        else if (m <= 8)         \
            RCBF_QPB_L(NN, 8);   \
        else if (m <= 12)        \
            RCBF_QPB_L(NN, 12);  \
        else                     \
            RCBF_QPB_L(NN, 16);  \
    } while (0)
    if (n == 1)
        RCBF_QPB_M(1);
    else if (n == 2)
        RCBF_QPB_M(2);
    else
        RCBF_QPB_M(3);
#undef RCBF_QPB_M
#undef RCBF_QPB_L
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
