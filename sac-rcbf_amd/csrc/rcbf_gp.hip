// rcbf_gp.hip -- GP disturbance posterior + C-ABI:
// rcbf_gp_predict = DynamicsModel.predict_disturbance with fitted GPs
// (rcbf_sac/dynamics.py:342-390, rcbf_sac/gp_model.py:86-114).
//
// One exact GP per state dimension i, all on the same training inputs:
//   k_i(x, x') = s_i exp(-|x - x'|^2 / (2 l_i^2))          (ScaleKernel(RBF))
//   mean_i(x)  = k_i(x, X) alpha_i,  alpha_i = (K_i + n_i I)^-1 y_i
//   var_i(x)   = s_i - k_i(x, X) (K_i + n_i I)^-1 k_i(X, x) + n_i  (likelihood noise)
// The host factors (K_i + n_i I)^-1 = R_i R_i^T (rank r; r = N is exact) and
// appends alpha_i as column r of Rt_i = [R_i | alpha_i | 0].  Then for a
// block of query rows b
//   Q_i(b, :) = k_i(b, X) Rt_i      -- a (B x N) (N x C) GEMM per GP
//   var = s_i + n_i - sum_{j<r} Q_i(b,j)^2,   mean = Q_i(b, r)
// k_i(b, X) is never stored: each wave builds its MFMA A-operand values
// in registers from the scaled inputs (|xq|^2 + |xt|^2 - 2 xq.xt, then exp),
// and the GEMM runs on the fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32
// products, the precision the reference's gpytorch model computes in).
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kGpRows = 128;   // query rows per workgroup
constexpr int kGpCols = 128;   // Rt columns per workgroup
constexpr int kGpChunk = 256;  // training rows staged in LDS at a time

// Workgroup (row tile, column block cb, GP i): 4 waves as 2 (rows) x 2 (cols),
// each wave a 64 x 64 output = 2 x 2 tiles of 32 x 32.
// partial[(i * n_cb + cb) * B + b] = sum over this block's columns j < r of Q^2;
// meanraw[i * B + b] = Q(b, r) from the block holding column r.
template <int D>
__global__ void __launch_bounds__(256) k_gp_qform(rcbf_gp_model m, int64_t B, const float* __restrict__ xq,
                                                  float* __restrict__ partial, float* __restrict__ meanraw) {
    constexpr int DP = (D + 3) / 4 * 4;  // LDS row stride (float4 reads)
    __shared__ float4 s_xt[kGpChunk * DP / 4];
    __shared__ float s_tn2[kGpChunk];
    __shared__ float s_rows[kGpRows];

    const int i = blockIdx.z;
    const int cb = blockIdx.y;
    const int n_cb = gridDim.y;
    const int64_t b0 = (int64_t)blockIdx.x * kGpRows;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int rw = (w >> 1) * 64, cw = (w & 1) * 64;
    const int half = lane >> 5, l32 = lane & 31;
    const float sl = m.inv_sl[i];
    const float s_i = m.outscale[i];

    // this lane's two query rows (A operand row = lane & 31 of each row tile)
    float xs[2][D], qn2[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        int64_t row = b0 + rw + t * 32 + l32;
        row = row < B ? row : B - 1;
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            // dynamics.py:376: test_x / train_x_std in fp64, then .float()
            float xn = (float)((double)xq[row * D + k] / m.x_std[k]);
            xs[t][k] = xn * sl;
            acc = fmaf(xs[t][k], xs[t][k], acc);
        }
        qn2[t] = acc;
    }

    f32x16 acc[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][c][r] = 0.0f;

    const float* xt_i = m.xt + (int64_t)i * m.N_pad * D;
    const float* tn2_i = m.tn2 + (int64_t)i * m.N_pad;
    const float* Rt_i = m.Rt + (int64_t)i * m.N_pad * m.C_pad + (int64_t)cb * kGpCols + cw + l32;

    for (int n0 = 0; n0 < m.N_pad; n0 += kGpChunk) {
        const int nch = min(kGpChunk, m.N_pad - n0);  // multiple of 32
        __syncthreads();
        for (int e = threadIdx.x; e < nch; e += 256) {
            float v[DP];
#pragma unroll
            for (int k = 0; k < DP; ++k) v[k] = k < D ? xt_i[(int64_t)(n0 + e) * D + k] : 0.0f;
#pragma unroll
            for (int q = 0; q < DP / 4; ++q) s_xt[e * (DP / 4) + q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
            s_tn2[e] = tn2_i[n0 + e];
        }
        __syncthreads();
        // B operand: Rt[n][col], n = k-step row of this half-wave
        const float* rp = Rt_i + (int64_t)(n0 + half) * m.C_pad;
        for (int k8 = 0; k8 < nch; k8 += 8)
#pragma unroll
        for (int kq = 0; kq < 8; kq += 2) {
            const int kk = k8 + kq;
            const int nl = kk + half;
            float bv0 = rp[(int64_t)kk * m.C_pad];
            float bv1 = rp[(int64_t)kk * m.C_pad + 32];
            float4 xt4[DP / 4];
#pragma unroll
            for (int q = 0; q < DP / 4; ++q) xt4[q] = s_xt[nl * (DP / 4) + q];
            const float* xtv = reinterpret_cast<const float*>(xt4);
            const float tn = s_tn2[nl];
            float av[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                float dot = 0.0f;
#pragma unroll
                for (int k = 0; k < D; ++k) dot = fmaf(xs[t][k], xtv[k], dot);
                float d2 = fmaxf(qn2[t] + tn - 2.0f * dot, 0.0f);
                av[t] = s_i * __expf(-d2);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                acc[t][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], bv0, acc[t][0], 0, 0, 0);
                acc[t][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], bv1, acc[t][1], 0, 0, 0);
            }
        }
    }

    // epilogue: C layout col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const int r_rank = m.r;
    float rs[2][16];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float v = 0.0f;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int col = cb * kGpCols + cw + c * 32 + l32;
                const float q = acc[t][c][r];
                v += (col < r_rank) ? q * q : 0.0f;
                if (col == r_rank) {
                    const int64_t row = b0 + rw + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                    if (row < B) meanraw[(int64_t)i * B + row] = q;
                }
            }
            rs[t][r] = v;
        }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float v = rs[t][r];
#pragma unroll
            for (int msk = 1; msk < 32; msk <<= 1) v += __shfl_xor(v, msk, 64);
            rs[t][r] = v;
        }
    // combine the two column-waves of each row half in a fixed order
    if ((w & 1) == 0 && l32 == 0) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) s_rows[rw + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * half] = rs[t][r];
    }
    __syncthreads();
    if ((w & 1) == 1 && l32 == 0) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int lr = rw + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                const int64_t row = b0 + lr;
                if (row < B) partial[((int64_t)i * n_cb + cb) * B + row] = s_rows[lr] + rs[t][r];
            }
    }
}

// mean/std (B, n_s) row-major like predict_disturbance's (n_test, n_s) output.
__global__ void __launch_bounds__(256) k_gp_finish(rcbf_gp_model m, int64_t B, int n_cb,
                                                   const float* __restrict__ partial,
                                                   const float* __restrict__ meanraw, float* __restrict__ mean_out,
                                                   float* __restrict__ std_out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= B * m.n_s) return;
    const int i = (int)(e % m.n_s);
    const int64_t b = e / m.n_s;
    float q = 0.0f;
    for (int c = 0; c < n_cb; ++c) q += partial[((int64_t)i * n_cb + c) * B + b];
    const float lat = fmaxf(m.outscale[i] - q, 0.0f);  // latent posterior variance
    const float var = lat + m.noise[i];                  // likelihood(model(x)).variance
    mean_out[e] = meanraw[(int64_t)i * B + b] * m.y_scale[i];
    std_out[e] = sqrtf(var) * m.y_scale[i];
}

}  // namespace

extern "C" {

int64_t rcbf_gp_workspace_floats(const rcbf_gp_model* m, int64_t B) {
    if (!m || B < 0) return -1;
    const int64_t n_cb = m->C_pad / kGpCols;
    return (int64_t)m->n_s * (n_cb + 1) * B;
}

int rcbf_gp_predict(const rcbf_gp_model* m, int64_t B, const float* x, float* mean_out, float* std_out,
                    float* workspace, hipStream_t stream) {
    if (!m) return RCBF_E_NULL;
    if (B < 0 || m->n_s < 1 || m->n_s > 10 || m->N < 1 || m->N_pad % 32 || m->N_pad < m->N || m->r < 1 ||
        m->r > m->N || m->C_pad % kGpCols || m->C_pad < m->r + 1)
        return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !mean_out || !std_out || !workspace || !m->xt || !m->tn2 || !m->Rt || !m->x_std || !m->inv_sl ||
        !m->outscale || !m->noise || !m->y_scale)
        return RCBF_E_NULL;
    const int n_cb = m->C_pad / kGpCols;
    float* partial = workspace;
    float* meanraw = workspace + (int64_t)m->n_s * n_cb * B;
    dim3 g((unsigned)((B + kGpRows - 1) / kGpRows), (unsigned)n_cb, (unsigned)m->n_s);
    switch (m->n_s) {  // D = n_s: the GP inputs are the full state
        case 3:
            hipLaunchKernelGGL((k_gp_qform<3>), g, dim3(256), 0, stream, *m, B, x, partial, meanraw);
            break;
        case 10:
            hipLaunchKernelGGL((k_gp_qform<10>), g, dim3(256), 0, stream, *m, B, x, partial, meanraw);
            break;
        default:
            return RCBF_E_BAD_SHAPE;
    }
    const int64_t tot = B * m->n_s;
    hipLaunchKernelGGL(k_gp_finish, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, *m, B, n_cb, partial,
                       meanraw, mean_out, std_out);
    return launch_status();
}

}  // extern "C"
