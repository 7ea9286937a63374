// rcbf_qp_bwd.hip -- generic QP backward + C-ABI: rcbf_qp_backward and
// rcbf_qp_backward_saved (the autograd of CBFQPLayer.solve_qp / cbf_layer,
// diff_cbf_qp.py:81-144, as qpth's QPFunction.backward).
#include "rcbf_qp_common.hpp"

using namespace rcbf;
using namespace rcbf_qp;

namespace {

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
// first maximal entry, d|x|/dx = sgn x).  Every output is [nullable]; the
// gradient rows leave through LDS with coalesced stores.
template <int N, int MP, bool DIAG>
__device__ __forceinline__ void qp_adjoint(const PMat<N, DIAG>& pm, const StagedQP<N, MP, float>& Q,
                                           const double* g, const QPResult<N, MP>& res, double* dz, double* eta,
                                           int* aidx) {
    double GA[N][N];
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
            for (int k = 0; k < N; ++k) GA[sl][k] = here ? (double)Q.G[r][k] : GA[sl][k];
            aidx[sl] = here ? r : aidx[sl];
        }
        nact += a ? 1 : 0;
    }
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
}

template <int N, int MP>
__global__ void __launch_bounds__(kQPBlock) k_qp_bwd(rcbf_params prm, int64_t B, int m, const float* __restrict__ P,
                                                     const float* __restrict__ q, const float* __restrict__ G,
                                                     const float* __restrict__ h, int normalize,
                                                     const float* __restrict__ grad_z, float* __restrict__ gP,
                                                     float* __restrict__ gq, float* __restrict__ gG,
                                                     float* __restrict__ gh, const double* __restrict__ z64_in) {
    extern __shared__ __align__(16) unsigned char qp_smem[];
    float* sG = reinterpret_cast<float*>(qp_smem);
    float* sh = sG + kQPBlock * odd_stride(m * N);
    float* sP = sh + kQPBlock * odd_stride(m);
    float* sq = sP + kQPBlock * odd_stride(N * N);
    const int64_t i0 = (int64_t)blockIdx.x * kQPBlock;
    const int nb = (int)((B - i0) < kQPBlock ? (B - i0) : kQPBlock);
    stage_in<float, MP * N>(G + i0 * m * N, sG, nb, m * N);
    stage_in<float, MP>(h + i0 * m, sh, nb, m);
    stage_in<float, N * N>(P + i0 * N * N, sP, nb, N * N);
    if (q) stage_in<float, N>(q + i0 * N, sq, nb, N);
    __syncthreads();
    const int lane = threadIdx.x;
    const bool active = lane < nb;
    const int64_t i = i0 + lane;
    StagedQP<N, MP, float> Q;
    float Nrm[MP];
    double rinv[MP];  // 1 / N_r from the normaliser
    int amax[MP];
    double g[N], z[N], dz[N], eta[N];
    int aidx[N];
    QPResult<N, MP> res;
    if (active) {
        staged_read<N, MP, float>(sG, sh, sP, sq, lane, m, q != nullptr, Q);
#pragma unroll
        for (int r = 0; r < MP; ++r) {
            float mx = fabsf(Q.G[r][0]);
            int a = 0;
#pragma unroll
            for (int k = 1; k < N; ++k) {
                bool gt = fabsf(Q.G[r][k]) > mx;
                a = gt ? k : a;
                mx = gt ? fabsf(Q.G[r][k]) : mx;
            }
            amax[r] = (fabsf(Q.h[r]) > mx) ? N : a;
            Nrm[r] = 1.0f;
        }
        if (normalize) normalize_rows<N, MP, float>(Q.G, Q.h, Nrm, nullptr, rinv);
#pragma unroll
        for (int a = 0; a < N; ++a) g[a] = (double)grad_z[i * N + a];
    } else {
        Q.diag = true;
    }
    if (__ballot(!Q.diag) == 0) {
        PMat<N, true> pm;
        double pd[N];
#pragma unroll
        for (int k = 0; k < N; ++k) pd[k] = active ? Q.P[k][k] : 1.0;
        pmat_set_diag_rt<N>(pm, pd);
        // The multipliers and the adjoint from ONE factorisation on the tight
        // rows of the optimum (structured_kkt_adjoint, diagonal P, q = 0),
        // where the optimum is the forward's saved fp64 solution (z64_in, what
        // qpth's QPFunction keeps for its backward) or, on the layer's own
        // rows, the closed-form one; a lane whose certificate fails re-solves
        // with Goldfarb-Idnani.
        bool need_gi = active;
        if (z64_in) {
            if (active && Q.qzero) {
#pragma unroll
                for (int k = 0; k < N; ++k) res.z[k] = z64_in[i * N + k];
                res.status = RCBF_QP_OK;
                need_gi = !structured_kkt_adjoint<N, MP, float>(Q, m, g, res, dz, eta, aidx);
            }
        } else if (__ballot(active && !layer_structured<N, MP, float>(Q, m)) == 0) {
            if (active) {
                structured_solve<N, MP, float>(Q, m, res.z, res.status);
                need_gi = !(res.status == RCBF_QP_OK &&
                            structured_kkt_adjoint<N, MP, float>(Q, m, g, res, dz, eta, aidx));
            }
        }
        if (need_gi) {
            gi_solve<N, MP, true, float>(pm, Q.q, Q.G, Q.h, 4 * (MP + N) + 8, res);
            qp_adjoint<N, MP, true>(pm, Q, g, res, dz, eta, aidx);
        }
    } else if (active) {
        PMat<N, false> pm;
        pmat_set_full<N>(pm, Q.P);
        if (!gi_solve_chol<N, MP, float>(Q, 4 * (MP + N) + 8, res))
            gi_solve<N, MP, false, float>(pm, Q.q, Q.G, Q.h, 4 * (MP + N) + 8, res);
        qp_adjoint<N, MP, false>(pm, Q, g, res, dz, eta, aidx);
    }
    __syncthreads();  // every lane is done reading the staged inputs: the buffers now carry the gradients
    if (active) {
#pragma unroll
        for (int k = 0; k < N; ++k) z[k] = res.z[k];
        const int wg = odd_stride(m * N), wh = odd_stride(m), wp = odd_stride(N * N), wq = odd_stride(N);
#pragma unroll
        for (int a = 0; a < N; ++a) {
            sq[lane * wq + a] = (float)dz[a];
#pragma unroll
            for (int b = 0; b < N; ++b) sP[lane * wp + a * N + b] = (float)(0.5 * (dz[a] * z[b] + z[a] * dz[b]));
        }
#pragma unroll
        for (int r = 0; r < MP; ++r) {
            if (r >= m) continue;
            double er = 0.0;
#pragma unroll
            for (int sl = 0; sl < N; ++sl) er = (aidx[sl] == r) ? eta[sl] : er;
            double gGn[N], ghn = -er;
#pragma unroll
            for (int k = 0; k < N; ++k) gGn[k] = er * z[k] + res.lam[r] * dz[k];
            double dN = 0.0, inr = 1.0;  // inr = 1 / N_r
            if (normalize) {
                inr = rinv[r];
                double acc = ghn * (double)Q.h[r];
#pragma unroll
                for (int k = 0; k < N; ++k) acc += gGn[k] * (double)Q.G[r][k];
                dN = -acc * inr;
            }
            auto sgn = [](float v) { return v > 0.0f ? 1.0 : (v < 0.0f ? -1.0 : 0.0); };
#pragma unroll
            for (int k = 0; k < N; ++k)
                sG[lane * wg + r * N + k] =
                    (float)(gGn[k] * inr + ((normalize && amax[r] == k) ? dN * sgn(Q.G[r][k]) : 0.0));
            sh[lane * wh + r] = (float)(ghn * inr + ((normalize && amax[r] == N) ? dN * sgn(Q.h[r]) : 0.0));
        }
    }
    __syncthreads();
    if (gG) stage_out<float>(gG + i0 * m * N, sG, nb, m * N);
    if (gh) stage_out<float>(gh + i0 * m, sh, nb, m);
    if (gP) stage_out<float>(gP + i0 * N * N, sP, nb, N * N);
    if (gq) stage_out<float>(gq + i0 * N, sq, nb, N);
}

}  // namespace

extern "C" {

int rcbf_qp_backward(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P, const float* q,
                     const float* G, const float* h, int32_t normalize, const float* grad_z, float* grad_P,
                     float* grad_q, float* grad_G, float* grad_h, hipStream_t stream) {
    return rcbf_qp_backward_saved(prm, B, n, m, P, q, G, h, normalize, nullptr, grad_z, grad_P, grad_q, grad_G, grad_h,
                                  stream);
}

int rcbf_qp_backward_saved(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P, const float* q,
                           const float* G, const float* h, int32_t normalize, const double* z64_saved,
                           const float* grad_z, float* grad_P, float* grad_q, float* grad_G, float* grad_h,
                           hipStream_t stream) {
    if (!prm) return RCBF_E_NULL;
    if (B < 0 || n < 1 || n > 3 || m < 1 || m > 16) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!P || !G || !h || !grad_z) return RCBF_E_NULL;
    // A PDIPM forward's saved point is an interior-point iterate (polished, but
    // not certified to the active-set tightness the one-factorisation backward
    // tests rows with): it could accept an incomplete active set, so that
    // backward re-solves exactly instead of starting from it.
    if (prm->solver == RCBF_SOLVER_PDIPM) z64_saved = nullptr;
    dim3 g((unsigned)((B + kQPBlock - 1) / kQPBlock)), b(kQPBlock);
    const size_t lds = (size_t)qp_lds_words(n, m) * sizeof(float);
#define RCBF_QPB_L(NN, MP)                                                                                       \
    hipLaunchKernelGGL((k_qp_bwd<NN, MP>), g, b, lds, stream, *prm, B, m, P, q, G, h, normalize, grad_z, grad_P, \
                       grad_q, grad_G, grad_h, z64_saved)
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
    if (n == 3 && m == 7)
        RCBF_QPB_L(3, 7);
    else if (n == 3 && m == 9)
        RCBF_QPB_L(3, 9);
    else if (n == 1)
        RCBF_QPB_M(1);
    else if (n == 2)
        RCBF_QPB_M(2);
    else
        RCBF_QPB_M(3);
#undef RCBF_QPB_M
#undef RCBF_QPB_L
    return launch_status();
}

}  // extern "C"
