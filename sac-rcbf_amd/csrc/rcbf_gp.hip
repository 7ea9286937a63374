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
// k_i(b, X) is never stored.  For every 32 training rows a wave forms the
// 32 x 32 exponent arguments of its 32 query rows with one small MFMA product
// over augmented vectors, then one exp2 per lane and k-step gives the A
// operand of the main product; [R | alpha] is staged once per workgroup in
// LDS.  Both products run on the fp32 MFMA (v_mfma_f32_32x32x2_f32, exact
// fp32 products, the precision the reference's gpytorch model computes in).
// For the exact posterior R = L^-T is upper triangular and the column block
// of logical columns [128 cb, 128 cb + 128) reads only training rows below
// 128 (cb + 1): half the work of the dense product (RCBF_GP_RT_UPPER).
#include <vector>
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kGpRows = 128;   // query rows per workgroup
constexpr int kGpCols = 128;   // Rt columns per workgroup
constexpr int kGpChunk = 256;  // training rows staged in LDS at a time
#ifndef RCBF_GP_SK_CHUNK
#define RCBF_GP_SK_CHUNK 256
#endif
// the split-K instantiation (small batches) stages fewer training rows at a time when
// RCBF_GP_SK_CHUNK < 256, so 4 workgroups fit a CU's LDS (study knob)
template <bool SK>
constexpr int gp_chunk() { return SK ? RCBF_GP_SK_CHUNK : kGpChunk; }
#ifndef RCBF_GP_DOT_MFMA
#define RCBF_GP_DOT_MFMA 1
#endif
// 1 (r04, the product): the arguments on the MFMA and [R | alpha] staged in
// LDS (gp_qform_dot_staged).  0: the earlier loop, kept for A/B builds: D VALU
// FMAs per A value and every wave loading its own B values.
constexpr bool kGpDot = RCBF_GP_DOT_MFMA != 0;
// 1: split-K launches k_gp_qform_sk2 (two wave groups, 512 threads); 0: k_gp_qform<D, 4, true> (256 threads)
#ifndef RCBF_GP_SK2
#define RCBF_GP_SK2 1
#endif
constexpr bool kGpSk2 = RCBF_GP_SK2 != 0 && kGpDot;
constexpr int kGpRtBuf = kGpDot ? 2 * 32 * kGpCols : 1;  // floats: two 32-row slices of the column block
template <int D>
struct GpAug {
    static constexpr int KA = (D + 2 + 1) / 2 * 2;    // [q0 | 1 | 2 L2E xs] . [1 | tn | xt], padded to even
    static constexpr int KS = KA / 2;                 // k-steps of the 32x32x2 product
    static constexpr int KSP = (KS + 3) / 4 * 4;      // per-half LDS stride (16-B reads)
    static constexpr int F4 = kGpDot ? 2 * KSP / 4 : (D + 3) / 4;  // float4s per staged training row
};

// This lane's B operand of the dot product: element 2 f + half of
// [q0, 1, 2 L2E xs, 0...].  The values pass through an empty asm first, so the
// half-select stays a select of two registers (folded into a select of two
// array slots it becomes a dynamic index, i.e. a scratch array).
template <int D>
__device__ __forceinline__ void gp_query_operand(const float (&xs2)[D], float q0, int half,
                                                 float (&qb)[GpAug<D>::KS]) {
    using A = GpAug<D>;
    float qa[A::KA];
#pragma unroll
    for (int e = 0; e < A::KA; ++e) {
        qa[e] = e == 0 ? q0 : (e == 1 ? 1.0f : (e - 2 < D ? xs2[e - 2] : 0.0f));
        asm volatile("" : "+v"(qa[e]));
    }
#pragma unroll
    for (int f = 0; f < A::KS; ++f) qb[f] = half ? qa[2 * f + 1] : qa[2 * f];
}

// The training loop (kGpDot).  Per block of 32 training rows t and the
// wave's 32 query rows b, one v_mfma_f32_32x32x2_f32 product over
//   arg(t, b) = [1, tn_t, xt_t] . [q0_b, 1, 2 L2E xs_b]
// (K = D + 2, padded to even: KS k-steps; q0 + tn first, then the D
// products, the order of the VALU chain it replaces) leaves arg(t, b) in the
// C layout: lane l, register r holds t = (r & 3) + 8 (r >> 2) + 4 (l >> 5),
// b = l & 31 -- exactly the A-operand layout of the main product's k-step r,
// so each k-step costs one fminf + exp2 per lane beside its 4 MFMAs, and the
// B operand of k-step r is Rt row t: rows 8 g + 4 half + j of the block in
// group g = r >> 2, j = r & 3.
// Block bg's 32 x 128 slice of Rt (16 KB) is
// copied to LDS buffer bg & 1 by the whole workgroup with 4 global_load_lds
// (16 B per lane, lane-linear: one wave-instruction = 2 rows) while block
// bg - 1 is computed; one barrier per block.  The k-step r B value of lane
// (l32, half) is then a ds_read_b128 of row 8 g + 4 half + j.
// G = 2 (the split-K instantiation, 512 threads): two groups of 4 waves share the workgroup's query rows
// and take alternate 32-row blocks (group g: blocks 2 it + g), two waves per SIMD, so one wave's LDS reads,
// exp2 and barrier waits overlap the other's MFMAs; the groups' accumulators are added through LDS after
// the loop (gp_qform_body).
template <int D, bool SK, bool HAS_MEAN, int G = 1>
__device__ __forceinline__ void gp_qform_dot_staged(const rcbf_gp_model& m, int i, int cb, int n_beg, int n_end,
                                                    const float (&xs2)[D], float q0, float log2s, const float* alpha_i,
                                                    const float* xt_i, const float* tn2_i, int64_t ldc, int half,
                                                    int l32, f32x16* acc, double& macc, float4* s_xt,
                                                    float* s_alpha, float* s_rt) {
    using A = GpAug<D>;
    constexpr float kL2E = 1.4426950408889634f;
    float* s_ta = reinterpret_cast<float*>(s_xt);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int grp = G == 1 ? 0 : w >> 2;  // wave group: blocks 2 it + grp
    float qb[A::KS];
    gp_query_operand<D>(xs2, q0, half, qb);
    const float* Rt_cb = m.Rt + (int64_t)i * m.N_pad * ldc + (int64_t)cb * kGpCols;  // this column block
    const int nb = (n_end - n_beg) / 32;  // N_pad and the split bounds are multiples of 32
    // G = 1: block bg -> buffer bg & 1.  G = 2: iteration it stages blocks 2 it, 2 it + 1 into buffers
    // 2 (it & 1), 2 (it & 1) + 1 (every thread copies 16 B of 4 slots of the 2 x 16 KB)
    auto issue_rt = [&](int it) {
#pragma unroll
        for (int gb = 0; gb < G; ++gb) {
            const int bg = G * it + gb;
            if (bg >= nb) break;
            float* buf = s_rt + (G * (it & 1) + gb) * 32 * kGpCols;
#pragma unroll
            for (int q = 0; q < 4 / G; ++q) {
                const int slot = q * (4 * G) + w;          // 64-lane slot of the 32 x 32 float4 image
                const int e = slot * 64 + lane;            // float4 index in it
                const float* src = Rt_cb + (int64_t)(n_beg + 32 * bg + (e >> 5)) * ldc + 4 * (e & 31);
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                                 (__attribute__((address_space(3))) void*)(buf + slot * 256),
                                                 16, 0, 0);
            }
        }
    };
    auto stage_ta = [&](int n0, int nch) {
        for (int e = threadIdx.x; e < nch; e += 256 * G) {
            float ta[A::KA];
            ta[0] = 1.0f;
            ta[1] = -kL2E * tn2_i[n0 + e];
#pragma unroll
            for (int k = 0; k < A::KA - 2; ++k) ta[2 + k] = k < D ? xt_i[(int64_t)(n0 + e) * D + k] : 0.0f;
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int f = 0; f < A::KSP; ++f) s_ta[e * 2 * A::KSP + h * A::KSP + f] = f < A::KS ? ta[2 * f + h] : 0.0f;
            if constexpr (HAS_MEAN) s_alpha[e] = alpha_i[(int64_t)(n0 + e) * ldc];
        }
    };
    const int nit = (nb + G - 1) / G;
    if (nb > 0) issue_rt(0);
#pragma unroll 1
    for (int it = 0; it < nit; ++it) {
        const int bg = G * it + grp;  // this wave's block
        const int lb0 = (G * it) % (gp_chunk<SK>() / 32);  // the iteration's first block within its chunk
        if (lb0 == 0) {  // a new chunk of training rows: every wave done with the previous one first
            __syncthreads();
            stage_ta(n_beg + 32 * G * it, min(gp_chunk<SK>(), n_end - (n_beg + 32 * G * it)));
        }
        // ONE barrier per iteration: its vmcnt(0) retires this wave's copies of iteration it, and past it
        // every wave has finished iteration it - 1, so its buffers are free for iteration it + 1
        __syncthreads();
        if (it + 1 < nit) issue_rt(it + 1);
        if (bg >= nb) continue;  // G = 2, odd block count: the second group sits out the last iteration
        const int lb = lb0 + grp;
        const float* buf = s_rt + (G * (it & 1) + grp) * 32 * kGpCols;
        const float* tp = s_ta + (lb * 32 + l32) * 2 * A::KSP + half * A::KSP;
        float af[A::KS];
#pragma unroll
        for (int f = 0; f < A::KS; ++f) af[f] = tp[f];
        f32x16 dd;
#pragma unroll
        for (int r = 0; r < 16; ++r) dd[r] = 0.0f;
#pragma unroll
        for (int f = 0; f < A::KS; ++f) dd = __builtin_amdgcn_mfma_f32_32x32x2f32(af[f], qb[f], dd, 0, 0, 0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            // keeps the LDS reads of a group (B values, alphas) from being hoisted over earlier groups
            // (registers: the kernel stays at 3 waves per SIMD)
            if constexpr (HAS_MEAN) asm volatile("" ::: "memory");
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 bq = reinterpret_cast<const float4*>(buf)[(8 * g + 4 * half + j) * 32 + l32];
                const float av = __builtin_amdgcn_exp2f(fminf(dd[4 * g + j], log2s));
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bq.x, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bq.y, acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bq.z, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bq.w, acc[3], 0, 0, 0);
                if constexpr (HAS_MEAN) macc = fma((double)av, (double)s_alpha[lb * 32 + 8 * g + 4 * half + j], macc);
            }
        }
    }
}

// Workgroup (row tile of 128 queries, column block cb of 128, GP i): wave w
// owns query rows 32w..32w+31 and all 128 columns (4 tiles of 32 x 32), so
// every A-operand value k_i(x_b, x_n) is built exactly once per workgroup and
// each wave reduces its own rows (no cross-wave combine).  Per k-step of 2
// training points a wave issues 4 MFMAs with one A value per lane
// (gp_qform_dot_staged; the level-0 loop builds it from D VALU FMAs + exp2
// and loads its own B values 4 k-steps ahead).
// partial[(i * n_cb + cb) * B + b] = sum over this block's columns j < r of Q^2;
// meanraw[i * B + b] = Q(b, r) from the block holding column r.
// Split-K (SK, small grids: few query tiles or a low-rank [R | alpha]):
// blockIdx.z = i * n_split + s and the workgroup sums only training rows
// [s per, (s + 1) per); it stores its raw Q tile to
// qraw[((i * n_split + s) * B + b) * C_pad + col] and k_gp_combine adds the
// n_split tiles (fixed order, deterministic) before squaring.
// The mean column (logical column r) of the single pass is not taken from
// the fp32 MFMA accumulator (one running sum over all N training rows: the
// large alternating alpha of an ill-conditioned fit made that chain lose
// 3e-4 of max|mean|).  Each lane instead adds its own A value times alpha_n
// (staged in LDS with the training rows) into an fp64 sum -- the products of two
// fp32 values are exact in fp64 -- and the two half-waves' sums are added in
// the epilogue.  One v_fma_f64 per k-step beside four MFMAs.
// MEAN: this workgroup's column block holds the mean column r (a separate
// instantiation, so the other ~95 % of the workgroups run the plain loop).
template <int D, int CT, bool SK, bool MEAN, int G = 1>
__device__ __forceinline__ void gp_qform_body(const rcbf_gp_model& m, int64_t B, const float* __restrict__ xq,
                                              float* __restrict__ partial, float* __restrict__ meanraw, int n_split,
                                              float* __restrict__ qraw, float4* s_xt, float* s_tn, float* s_alpha,
                                              float* s_rt) {
    constexpr int DP = (D + 3) / 4 * 4;  // LDS row stride (float4 reads)
    constexpr float kL2E = 1.4426950408889634f;
    // gp_qform_dot_staged accumulates the 4 column tiles of a whole 128-column block (acc[0..3] from one
    // ds_read_b128 of B values) and does not read `sub`: only CT = 4 is correct on that path
    static_assert(!kGpDot || CT == 4, "the MFMA-argument path (RCBF_GP_DOT_MFMA) needs CT == 4");

    // CT column tiles of 32 per wave: 4 (the whole 128-column block) or 2
    // (half of it, twice the workgroups for small query batches)
    const int i = SK ? (int)blockIdx.z / n_split : (int)blockIdx.z;
    const int split = SK ? (int)blockIdx.z % n_split : 0;
    const int cb = blockIdx.y / (4 / CT);          // 128-column block
    const int sub = blockIdx.y % (4 / CT);         // which CT tiles of it
    const int n_part = gridDim.y;
    static_assert(G == 1 || (G == 2 && SK && kGpDot), "two wave groups: the split-K MFMA-argument path only");
    const int64_t b0 = (int64_t)blockIdx.x * kGpRows;
    const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) & 3;  // w: the wave's 32 query rows
    const int grp = G == 1 ? 0 : (int)(threadIdx.x >> 8);           // wave group (G = 2)
    const int half = lane >> 5, l32 = lane & 31;
    const float sl = m.inv_sl[i];
    const float log2s = __log2f(m.outscale[i]);

    // A(b, n) = s exp(-|xs_b - xt_n|^2) = exp2(log2 s - L2E |xs|^2 - L2E |xt|^2 + 2 L2E xs.xt)
    float xs2[D], q0;
    {
        int64_t row = b0 + 32 * w + l32;
        row = row < B ? row : B - 1;
        float nrm = 0.0f;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            // dynamics.py:376: test_x / train_x_std in fp64, then .float()
            const float xs = (float)((double)xq[row * D + k] / m.x_std[k]) * sl;
            nrm = fmaf(xs, xs, nrm);
            xs2[k] = 2.0f * kL2E * xs;
        }
        q0 = fmaf(-kL2E, nrm, log2s);
    }

    f32x16 acc[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][r] = 0.0f;

    const float* xt_i = m.xt + (int64_t)i * m.N_pad * D;
    const float* tn2_i = m.tn2 + (int64_t)i * m.N_pad;
    const int64_t ldc = m.C_pad;
    // Rt columns are stored lane-interleaved per 128-column block (physical
    // 4 l + c holds logical column 32 c + l), so one dwordx4 load gives a lane
    // its B values for the 4 column tiles.
    const float* Rt_i = m.Rt + (int64_t)i * m.N_pad * ldc + (int64_t)cb * kGpCols + 4 * l32 + CT * sub;

    // exact posterior: R = L^-T, so logical column j has no nonzero row past j and this block's columns
    // (< 128 (cb + 1)) read only the training rows below that (the alpha column r = N sits in the last
    // block, whose bound is >= N_pad).  Half the MFMA work and the Rt traffic of the dense product.
    const int k_end = (m.flags & RCBF_GP_RT_UPPER) ? min(m.N_pad, (cb + 1) * kGpCols) : m.N_pad;
    int n_beg = 0, n_end = k_end;
    if constexpr (SK) {  // this block's rows in n_split equal parts (multiples of 32)
        const int per = ((k_end + n_split - 1) / n_split + 31) / 32 * 32;
        n_beg = min(k_end, split * per);
        n_end = min(k_end, n_beg + per);
    }
    // does this workgroup hold the mean column r (uniform)?  alpha_n = Rt[n][r] sits at the physical
    // column of logical column r (128-column blocks, lane-interleaved: 4 l + c holds 32 c + l)
    const int r_rank = m.r;
    const int mcol = r_rank - (cb * kGpCols + 32 * CT * sub);
    constexpr bool has_mean = MEAN && !SK;
    (void)mcol;
    const int64_t alpha_phys = (int64_t)(r_rank / kGpCols) * kGpCols + 4 * ((r_rank % kGpCols) % 32) +
                               (r_rank % kGpCols) / 32;
    const float* alpha_i = m.Rt + (int64_t)i * m.N_pad * ldc + alpha_phys;
    double macc = 0.0;
    if constexpr (kGpDot) {
        gp_qform_dot_staged<D, SK, has_mean, G>(m, i, cb, n_beg, n_end, xs2, q0, log2s, alpha_i, xt_i, tn2_i, ldc,
                                                half, l32, acc, macc, s_xt, s_alpha, s_rt);
        if constexpr (G == 2) {  // group 1 hands its accumulators to group 0 through LDS (the staging buffers)
            __syncthreads();
            // element-major: register (c, r) of the 256 lanes of a group is one contiguous row of 256 floats,
            // so every LDS access is lane-consecutive (no bank conflicts); 64 KB = the four staging buffers
            float* xa = s_rt + w * 64 + lane;
            if (grp == 1) {
#pragma unroll
                for (int c = 0; c < CT; ++c)
#pragma unroll
                    for (int r = 0; r < 16; ++r) xa[(c * 16 + r) * 256] = acc[c][r];
            }
            __syncthreads();
            if (grp == 1) return;
#pragma unroll
            for (int c = 0; c < CT; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[c][r] += xa[(c * 16 + r) * 256];
        }
    } else
    for (int n0 = n_beg; n0 < n_end; n0 += kGpChunk) {
        const int nch = min(kGpChunk, n_end - n0);  // multiple of 32
        __syncthreads();
        for (int e = threadIdx.x; e < nch; e += 256) {
            float v[DP];
#pragma unroll
            for (int k = 0; k < DP; ++k) v[k] = k < D ? xt_i[(int64_t)(n0 + e) * D + k] : 0.0f;
#pragma unroll
            for (int q = 0; q < DP / 4; ++q)
                s_xt[e * (DP / 4) + q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
            s_tn[e] = -kL2E * tn2_i[n0 + e];
            if constexpr (!SK) {
                if (has_mean) s_alpha[e] = alpha_i[(int64_t)(n0 + e) * ldc];
            }
        }
        __syncthreads();
        // B operand of k-step kk: Rt[n0 + kk + half][cb*128 + 32c + l32]
        const float* rp = Rt_i + (int64_t)(n0 + half) * ldc;
        float bcur[4][CT], bnx[4][CT];
        auto ldb = [&](int k, float* dst) {
            if constexpr (CT == 4) {
                const float4 v = *reinterpret_cast<const float4*>(rp + (int64_t)k * ldc);
                dst[0] = v.x, dst[1] = v.y, dst[2] = v.z, dst[3] = v.w;
            } else {
                const float2 v = *reinterpret_cast<const float2*>(rp + (int64_t)k * ldc);
                dst[0] = v.x, dst[1] = v.y;
            }
        };
#pragma unroll
        for (int q = 0; q < 4; ++q) ldb(2 * q, bcur[q]);
        for (int k8 = 0; k8 < nch; k8 += 8) {
            const bool more = k8 + 8 < nch;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (more)
                    ldb(k8 + 8 + 2 * q, bnx[q]);
                else
#pragma unroll
                    for (int c = 0; c < CT; ++c) bnx[q][c] = 0.0f;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int nl = k8 + 2 * q + half;
                float4 xt4[DP / 4];
#pragma unroll
                for (int u = 0; u < DP / 4; ++u) xt4[u] = s_xt[nl * (DP / 4) + u];
                const float* xtv = reinterpret_cast<const float*>(xt4);
                float arg = q0 + s_tn[nl];
#pragma unroll
                for (int k = 0; k < D; ++k) arg = fmaf(xs2[k], xtv[k], arg);
                const float av = __builtin_amdgcn_exp2f(fminf(arg, log2s));
#pragma unroll
                for (int c = 0; c < CT; ++c)
                    acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bcur[q][c], acc[c], 0, 0, 0);
                if constexpr (!SK) {
                    if (has_mean) macc = fma((double)av, (double)s_alpha[nl], macc);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int c = 0; c < CT; ++c) bcur[q][c] = bnx[q][c];
        }
    }

    // epilogue: C layout col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    if constexpr (SK) {
        float* qt = qraw + ((int64_t)i * n_split + split) * B * ldc;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t row = b0 + 32 * w + (r & 3) + 8 * (r >> 2) + 4 * half;
            if (row < B) {
#pragma unroll
                for (int c = 0; c < CT; ++c) qt[row * ldc + cb * kGpCols + 32 * (c + CT * sub) + l32] = acc[c][r];
            }
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t row = b0 + 32 * w + (r & 3) + 8 * (r >> 2) + 4 * half;
        float v = 0.0f;
#pragma unroll
        for (int c = 0; c < CT; ++c) {
            const int col = cb * kGpCols + 32 * (c + CT * sub) + l32;
            const float q = acc[c][r];
            v += (col < r_rank) ? q * q : 0.0f;
        }
#pragma unroll
        for (int msk = 1; msk < 32; msk <<= 1) v += __shfl_xor(v, msk, 64);
        if (l32 == 0 && row < B) partial[((int64_t)i * n_part + blockIdx.y) * B + row] = v;
    }
    if constexpr (has_mean) {  // lane (l32, half) summed row b0 + 32 w + l32 over the training rows of parity half
        const double tot = macc + __shfl_xor(macc, 32, 64);
        const int64_t row = b0 + 32 * w + l32;
        if (half == 0 && row < B) meanraw[(int64_t)i * B + row] = (float)tot;
    }
}

template <int D, int CT, bool SK = false>
__global__ void __launch_bounds__(256) k_gp_qform(rcbf_gp_model m, int64_t B, const float* __restrict__ xq,
                                                  float* __restrict__ partial, float* __restrict__ meanraw,
                                                  int n_split = 1, float* __restrict__ qraw = nullptr) {
    __shared__ float4 s_xt[(kGpDot ? gp_chunk<SK>() : kGpChunk) * GpAug<D>::F4];
    __shared__ float s_tn[kGpDot ? 1 : kGpChunk];
    __shared__ float s_alpha[SK ? 1 : kGpChunk];
    __shared__ __attribute__((aligned(16))) float s_rt[kGpRtBuf];
    const int mcol = m.r - ((int)(blockIdx.y / (4 / CT)) * kGpCols + 32 * CT * (int)(blockIdx.y % (4 / CT)));
    if (!SK && mcol >= 0 && mcol < 32 * CT)  // uniform: the block holding the mean column
        gp_qform_body<D, CT, SK, true>(m, B, xq, partial, meanraw, n_split, qraw, s_xt, s_tn, s_alpha, s_rt);
    else
        gp_qform_body<D, CT, SK, false>(m, B, xq, partial, meanraw, n_split, qraw, s_xt, s_tn, s_alpha, s_rt);
}

// The split-K instantiation with two wave groups (G = 2, 512 threads): each 128-query workgroup runs 8
// waves, two per SIMD, over alternate 32-row blocks of its split (gp_qform_dot_staged), four staging
// buffers (64 KB, reused for the groups' accumulator hand-off).
template <int D>
__global__ void __launch_bounds__(512) k_gp_qform_sk2(rcbf_gp_model m, int64_t B, const float* __restrict__ xq,
                                                      float* __restrict__ partial, float* __restrict__ meanraw,
                                                      int n_split, float* __restrict__ qraw) {
    __shared__ float4 s_xt[gp_chunk<true>() * GpAug<D>::F4];
    __shared__ float s_tn[1];
    __shared__ float s_alpha[1];
    __shared__ __attribute__((aligned(16))) float s_rt[2 * kGpRtBuf];
    gp_qform_body<D, 4, true, false, 2>(m, B, xq, partial, meanraw, n_split, qraw, s_xt, s_tn, s_alpha, s_rt);
}

// Few queries (B <= 8, the per-env-step query of main.py, B = 1): the
// posterior is a GEMV per GP, bound by streaming [R | alpha] (rank 100:
// 10 x 3008 x 128 fp32 = 15.4 MB), so it skips the MFMA tiles (127 of 128
// query rows would be padding).  ONE launch, r05:
//  * tile = (GP i, 128-column block cb, 64 training rows): 32 KB, every row
//    one whole 512-B line pair; thread t streams rows (t >> 5) + 8 j, j < 8,
//    float4 t & 31, its 8 loads issued together with the tile's training rows
//    and queries, so the tile pays one memory round trip; the kernel values
//    k_i(x_b, x_n) of its rows go through LDS.  The exact factor
//    (RCBF_GP_RT_UPPER) only has tiles below 128 (cb + 1).  Rank 100:
//    10 x 47 = 470 workgroups; exact N = 3000: 5 990.
//  * the 128 x BQ partial of a tile goes to the workspace; the last tile of
//    block (i, cb) to finish (a per-block arrival counter) sums the block's
//    partials in a fixed order (deterministic whichever tile is last), forms
//    sum_{j < r} Q^2 and the mean column, and -- when the GP has one column
//    block (a Lanczos factor) -- writes mean and std; otherwise the last
//    block of GP i to finish (a per-GP counter) does.  No combine or finish
//    launch.
// The counters live in the first words of the workspace, zero before the
// first call (the caller zero-fills a new workspace) and reset to zero by the
// workgroups that consume them.  Hand-off (cdna_hip_programming.md §6 G16,
// MI355X_MICROARCH.md "Valid forms", row 1): every handed-off byte is stored
// `sc1` (write-through, 16-B tile partials / 4-B block sums), every storing
// wave drains its stores (`s_waitcnt vmcnt(0)`) before the workgroup barrier
// behind which ONE lane adds to the arrival counter (relaxed, agent scope),
// and the workgroup whose add returned the last ticket reads every handed-off
// byte with `sc1` loads.  No __threadfence: an agent-scope release writes back
// the whole XCD L2 and an acquire invalidates the CU's L1 (r05b, with them in
// every workgroup: 72 us for rank 100 at B = 1).
#ifndef RCBF_GV_ROWS
#define RCBF_GV_ROWS 64
#endif
constexpr int kGvRows = RCBF_GV_ROWS;  // training rows per tile (a tile spans a whole 128-column block)

// tiles of one GP, and where column block cb's tiles start
__host__ __device__ inline int gp_gv_kend(const rcbf_gp_model& m, int cb) {
    return (m.flags & RCBF_GP_RT_UPPER) ? min(m.N_pad, kGpCols * (cb + 1)) : m.N_pad;
}
__host__ __device__ inline int gp_gv_rowtiles(const rcbf_gp_model& m, int cb) {
    return (gp_gv_kend(m, cb) + kGvRows - 1) / kGvRows;
}
inline int gp_gv_tiles(const rcbf_gp_model& m) {
    int t = 0;
    for (int cb = 0; cb < m.C_pad / kGpCols; ++cb) t += gp_gv_rowtiles(m, cb);
    return t;
}
// counter words at the start of the workspace: n_s * n_cb block counters, then n_s GP counters, each
// on a 128-B line of its own -- arrivals on one line serialise at the memory-side atomic unit (~13 ns
// each): with the 10 GPs' counters in one line, rank 100 at B = 1 spent ~13 us of its 18 there (r05e)
// The line after them holds the hand-off's fail word: a workgroup whose ticket is past its block's (or
// GP's) arrival count proves the counter was not zero when the call started (a workspace that was not
// zero-filled, a call aborted part-way, or two calls sharing one workspace at once) and sets bit 0;
// rcbf_gp_workspace_check reports it and zeroes the counters.
constexpr int kGvCtrStride = 32;  // words
__host__ __device__ inline int64_t gp_fail_word(const rcbf_gp_model& m) {
    return (int64_t)m.n_s * (m.C_pad / kGpCols + 1) * kGvCtrStride;
}
// the line after the fail word: the all-GPs arrival counter of the fused safe action (k_gp_gemv_sa)
__host__ __device__ inline int64_t gp_sa_word(const rcbf_gp_model& m) { return gp_fail_word(m) + kGvCtrStride; }
inline int64_t gp_counter_words(const rcbf_gp_model& m) { return gp_fail_word(m) + 2 * kGvCtrStride; }

struct GpCols {
    int32_t n;
    int32_t idx[10];
};

// The fused RCBF_SAC.get_safe_action of one observation with the GP posterior
// (k_gp_gemv_sa): what the last workgroup to finish reads and writes.
struct GpSafeAction {
    rcbf_params prm;
    const float* obs;      // (B, n_o) f32 observation rows: the GP query is get_state(obs)
    const float* u_rl;     // (B, n_u) f32 policy actions
    float* hmean;          // workspace hand-off of the posterior: (n_s, BQ) mean, std (sc1)
    float* hstd;
    float* u_out;          // [nullable] (B, n_u) f32 device
    float* u_host;         // [nullable] (B, n_u) f32 pinned host memory
    uint32_t* done_word;   // [nullable] pinned host completion word
    int32_t* status_out;   // [nullable]
    int32_t* fail_flag;    // [nullable]
    uint32_t seq;
};

// the hand-off's loads and 4-B stores: relaxed agent-scope atomics lower to global_load/store ... sc1
__device__ __forceinline__ float ld_sc1(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ticket(unsigned* c) {
    return __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// sum_{r < n} p[r * stride] in order r = 0, 1, ... with sc1 loads, 48 in flight at a time (a load used
// at once would cost a full memory round trip per term: r05c, 24 terms ~ 20 us)
__device__ __forceinline__ float sum_sc1(const float* p, int n, int64_t stride) {
    constexpr int kBatch = 48;
    float q = 0.0f;
    for (int r0 = 0; r0 < n; r0 += kBatch) {
        float a[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) a[u] = ld_sc1(p + (int64_t)min(r0 + u, n - 1) * stride);
#pragma unroll
        for (int u = 0; u < kBatch; ++u) q += (r0 + u < n) ? a[u] : 0.0f;
    }
    return q;
}

// mean and std of GP i at query b from q = sum_{j < r} Q^2 and the mean column's raw value (the
// arithmetic of gp_mean_std, dynamics.py:371-380 after gpytorch), into the row and column outputs
// (os, nz, ys: GP i's outputscale, noise and y_scale, loaded at the kernel's start, off the tail)
__device__ __forceinline__ void gp_gv_finish(const rcbf_gp_model& m, int64_t B, int i, int b, float q, float mraw,
                                             float os, float nz, float ys, float* mean_out, float* std_out,
                                             const GpCols& cols, float* mean_cols, float* std_cols,
                                             float* hmean = nullptr, float* hstd = nullptr, int bq = 1) {
    const float lat = fmaxf(os - q, 0.0f);  // latent posterior variance
    const float var = lat + nz;             // likelihood(model(x)).variance
    const float mu = mraw * ys;
    const float sd = sqrtf(var) * ys;
    if (mean_out) mean_out[(int64_t)b * m.n_s + i] = mu;
    if (std_out) std_out[(int64_t)b * m.n_s + i] = sd;
    if (hmean) {  // the fused safe action's hand-off (write-through, read with sc1 loads)
        st_sc1(hmean + (int64_t)i * bq + b, mu);
        st_sc1(hstd + (int64_t)i * bq + b, sd);
    }
    for (int c = 0; c < cols.n; ++c) {
        if (cols.idx[c] == i) {
            if (mean_cols) mean_cols[(int64_t)c * B + b] = mu;
            if (std_cols) std_cols[(int64_t)c * B + b] = sd;
        }
    }
}

// The fused safe action's last stage (k_gp_gemv_sa), run by every workgroup that finished a GP: its
// mean / std went out write-through and drained, then an arrival at the all-GPs counter; the last of the
// n_s finishers forms RCBF_SAC.get_safe_action for its query rows from the handed-off posterior -- the
// state from the observation, the CBF rows, the exact QP, the clamp (the arithmetic of
// rcbf_obs_safe_action, so the result equals the three-launch path bit for bit) -- writes the action to
// the device and / or pinned host memory, and publishes the completion word system-wide.
template <int BQ, int SAM, int SAK>
__device__ __forceinline__ void gp_sa_finish(const rcbf_gp_model& m, int64_t B, unsigned* counters,
                                             const GpSafeAction& sa) {
    __shared__ int s_all;
    const int t = threadIdx.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        const unsigned tk = ticket(&counters[gp_sa_word(m)]);
        if (tk >= (unsigned)m.n_s) atomicOr(&counters[gp_fail_word(m)], 1u);
        s_all = tk == (unsigned)(m.n_s - 1);
    }
    __syncthreads();
    if (!s_all) return;
    using DD = Dims<SAM, SAK>;
    if (t < B) {
        constexpr int NO = Dims<SAM, 1>::NO;
        float o[NO], xs[DD::NS], us[DD::NU], mm[DD::NS], ss[DD::NS], uf[DD::NU];
#pragma unroll
        for (int k = 0; k < DD::NS; ++k) {
            mm[k] = ld_sc1(sa.hmean + k * BQ + t);
            ss[k] = ld_sc1(sa.hstd + k * BQ + t);
        }
#pragma unroll
        for (int k = 0; k < NO; ++k) o[k] = sa.obs[(int64_t)t * NO + k];
#pragma unroll
        for (int c = 0; c < DD::NU; ++c) us[c] = sa.u_rl[(int64_t)t * DD::NU + c];
        state_from_obs32<SAM>(o, xs);
        LayerState<SAM, SAK> L;
        layer_forward<RCBF_SOLVER_ACTIVE_SET, SAM, SAK>(sa.prm, xs, us, mm, ss, uf, L);
#pragma unroll
        for (int c = 0; c < DD::NU; ++c) {
            if (sa.u_out) sa.u_out[(int64_t)t * DD::NU + c] = uf[c];
            if (sa.u_host) sa.u_host[(int64_t)t * DD::NU + c] = uf[c];
        }
        report(L.qp.status, sa.status_out, t, sa.fail_flag);
    }
    __syncthreads();
    if (t == 0) {
        atomicExch(&counters[gp_sa_word(m)], 0u);  // consumed: zero for the next call
        if (sa.done_word) {
            __threadfence_system();  // the action (and every status word) lands before the word
            __hip_atomic_store(sa.done_word, sa.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// SAM < 0: the GP posterior alone (k_gp_gemv); SAM = mode, SAK = hazards: the fused safe action
// (k_gp_gemv_sa, BQ = 1), whose query is get_state(obs) formed in every workgroup.
template <int D, int BQ, int SAM = -1, int SAK = 1>
__device__ __forceinline__ void gp_gemv_body(const rcbf_gp_model& m, int64_t B, const float* __restrict__ xq,
                                             int T, unsigned* counters, float* part, float* blk, float* meanraw,
                                             float* __restrict__ mean_out, float* __restrict__ std_out,
                                             const GpCols& cols, float* __restrict__ mean_cols,
                                             float* __restrict__ std_cols, const GpSafeAction* sa) {
    constexpr bool kSA = SAM >= 0;
    float* hmean = nullptr;
    float* hstd = nullptr;
    if constexpr (kSA) {
        hmean = sa->hmean;
        hstd = sa->hstd;
    }
    constexpr float kL2E = 1.4426950408889634f;
    constexpr int RJ = kGvRows / 8;  // rows per thread
    __shared__ float s_xs[BQ][D];
    __shared__ float s_k[BQ][kGvRows];
    __shared__ float4 s_red[4][BQ][32];
    __shared__ float s_bsum[4][BQ];
    __shared__ float s_half[2][kGpCols];
    __shared__ float s_mean[BQ];
    __shared__ int s_last;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int i = blockIdx.y;
    const int n_cb = m.C_pad / kGpCols;
    // tile -> (cb, rc); tiles are cb-major, then row tile
    int rc = blockIdx.x, cb = 0, base = 0;
    int nrc = gp_gv_rowtiles(m, 0);
    while (rc >= nrc) {
        rc -= nrc;
        base += nrc;
        ++cb;
        nrc = gp_gv_rowtiles(m, cb);
    }
    const int n0 = rc * kGvRows;
    const int nrows = min(kGvRows, gp_gv_kend(m, cb) - n0);  // a multiple of 32
    const int64_t ldc = m.C_pad;

    // 1. every load of the tile at once -- this thread's 128 B of Rt, then its training row (t < 64)
    //    and query component (t < BQ D) -- so the whole tile pays one memory round trip.  Rows past
    //    the tile's end re-read row n0 (in bounds) and get a zero kernel value.  Default-policy loads:
    //    the factor is re-read by every query until the next refit, and back-to-back calls gain from
    //    what the caches keep (r05u: B = 1 / 2 / 8 6.29 / 7.30 / 16.4 us with nt, 6.20 / 7.06 / 15.6 without).
    const float* Rp = m.Rt + ((int64_t)i * m.N_pad + n0) * ldc + cb * kGpCols + 4 * (t & 31);
    f32x4 v[RJ];
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        const int rr = (t >> 5) + 8 * j;
        v[j] = *reinterpret_cast<const f32x4*>(Rp + (int64_t)(rr < nrows ? rr : 0) * ldc);
    }
    const float sl = m.inv_sl[i];
    const float os = m.outscale[i], nz = m.noise[i], ys = m.y_scale[i];
    const float log2s = __log2f(os);
    float xt[D], tn = 0.0f;
    {
        const int n = n0 + (t < nrows ? t : 0);
#pragma unroll
        for (int k = 0; k < D; ++k) xt[k] = m.xt[((int64_t)i * m.N_pad + n) * D + k];
        tn = -kL2E * m.tn2[(int64_t)i * m.N_pad + n];
    }
    float xs_raw = 0.0f;
    double xstd = 1.0;
    if (t < BQ * D) {
        const int b = t / D, k = t % D;
        const int64_t row = b < B ? b : B - 1;
        if constexpr (kSA) {  // the query state get_state(obs) (dynamics.py:190-232), as rcbf_state_from_obs forms it
            constexpr int NO = Dims<(kSA ? SAM : 0), 1>::NO;
            float o[NO], st[Dims<(kSA ? SAM : 0), 1>::NS];
#pragma unroll
            for (int kk = 0; kk < NO; ++kk) o[kk] = sa->obs[row * NO + kk];
            state_from_obs32<(kSA ? SAM : 0)>(o, st);
            xs_raw = st[k];
        } else {
            xs_raw = xq[row * D + k];
        }
        xstd = m.x_std[k];
    }
    // 2. the scaled queries (dynamics.py:376: test_x / train_x_std in fp64, then .float()).  The barriers
    //    here are raw s_barrier with an LDS drain only: __syncthreads() would also drain vmcnt, i.e. wait
    //    for the Rt loads.
    if (t < BQ * D) s_xs[t / D][t % D] = (float)((double)xs_raw / xstd) * sl;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // 3. k_i(x_b, x_n) of the tile's rows (the arithmetic of k_gp_qform's level-0 loop)
    if (t < kGvRows) {
#pragma unroll
        for (int b = 0; b < BQ; ++b) {
            float kv = 0.0f;
            if (t < nrows) {
                float nrm = 0.0f;
#pragma unroll
                for (int k = 0; k < D; ++k) nrm = fmaf(s_xs[b][k], s_xs[b][k], nrm);
                float arg = fmaf(-kL2E, nrm, log2s) + tn;
#pragma unroll
                for (int k = 0; k < D; ++k) arg = fmaf(2.0f * kL2E * s_xs[b][k], xt[k], arg);
                kv = __builtin_amdgcn_exp2f(fminf(arg, log2s));
            }
            s_k[b][t] = kv;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // 4. this thread's rows into 4 columns x BQ queries
    float4 acc[BQ];
#pragma unroll
    for (int b = 0; b < BQ; ++b) acc[b] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
#pragma unroll
        for (int b = 0; b < BQ; ++b) {
            const float kv = s_k[b][(t >> 5) + 8 * j];
            acc[b].x = fmaf(kv, v[j][0], acc[b].x);
            acc[b].y = fmaf(kv, v[j][1], acc[b].y);
            acc[b].z = fmaf(kv, v[j][2], acc[b].z);
            acc[b].w = fmaf(kv, v[j][3], acc[b].w);
        }
    }
#if defined(RCBF_GV_STUDY) && RCBF_GV_STUDY == 3  // study: the tile's loads and FMAs only
    {
        float z = 0.0f;
#pragma unroll
        for (int b = 0; b < BQ; ++b) z += acc[b].x + acc[b].y + acc[b].z + acc[b].w;
        if (z == 1.2345f) part[t] = z;
    }
    return;
#endif
    // 5. sum the wave's two row groups (lane bit 5), then the 4 waves through LDS
#pragma unroll
    for (int b = 0; b < BQ; ++b) {
        acc[b].x += __shfl_xor(acc[b].x, 32, 64);
        acc[b].y += __shfl_xor(acc[b].y, 32, 64);
        acc[b].z += __shfl_xor(acc[b].z, 32, 64);
        acc[b].w += __shfl_xor(acc[b].w, 32, 64);
    }
    if (lane < 32) {
#pragma unroll
        for (int b = 0; b < BQ; ++b) s_red[w][b][lane] = acc[b];
    }
    __syncthreads();
    const int tile = base + rc;
    if (t < 32 * BQ) {
        const int b = t >> 5, f = t & 31;
        float4 a = s_red[0][b][f];
#pragma unroll
        for (int u = 1; u < 4; ++u) {
            const float4 o = s_red[u][b][f];
            a.x += o.x, a.y += o.y, a.z += o.z, a.w += o.w;
        }
        st_out4<true>(part + (((int64_t)i * T + tile) * BQ + b) * kGpCols + 4 * f, a);  // sc1
    }
#if defined(RCBF_GV_STUDY) && RCBF_GV_STUDY == 1  // study: no hand-off (partials stored, no arrival)
    return;
#endif
    // 6. arrival at block (i, cb): the last of its tiles reduces the block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        const unsigned tk = ticket(&counters[(i * n_cb + cb) * kGvCtrStride]);
        if (tk >= (unsigned)nrc) atomicOr(&counters[gp_fail_word(m)], 1u);  // the counter was not zero at entry
        s_last = tk == (unsigned)(nrc - 1);
    }
    __syncthreads();
    if (!s_last) return;
    const int r_rank = m.r;
    // thread t: physical column p = t & 127 of the block (4-B sc1 loads, a wave instruction reads two whole
    // lines).  BQ = 1: the workgroup's halves sum the even and the odd tiles, added in that order through LDS;
    // a tile's half depends on its index alone, so the exact-zero tiles a dense pass adds past an upper
    // factor's block change no sum.  BQ > 1: half t >> 7 takes queries b = (t >> 7), (t >> 7) + 2, ...
    const int p = t & 127;
    const int lc = cb * kGpCols + 32 * (p & 3) + (p >> 2);  // logical column (4 l + c holds 32 c + l)
    float vq[(BQ + 1) / 2];
    if constexpr (BQ == 1) {
        const int g = t >> 7, ng = (nrc - g + 1) / 2;
        s_half[g][p] = ng > 0 ? sum_sc1(part + ((int64_t)i * T + base + g) * kGpCols + p, ng, 2 * kGpCols) : 0.0f;
        __syncthreads();
        const float q = s_half[0][p] + s_half[1][p];
        if (t < kGpCols && lc == r_rank) {
            st_sc1(meanraw + (int64_t)i * BQ, q);
            s_mean[0] = q;
        }
        vq[0] = (t < kGpCols && lc < r_rank) ? q * q : 0.0f;
    } else {
#pragma unroll
        for (int h = 0; h < (BQ + 1) / 2; ++h) {
            const int b = (t >> 7) + 2 * h;
            float q = 0.0f;
            if (b < BQ) {
                q = sum_sc1(part + (((int64_t)i * T + base) * BQ + b) * kGpCols + p, nrc, (int64_t)BQ * kGpCols);
                if (lc == r_rank && b < B) {
                    st_sc1(meanraw + (int64_t)i * BQ + b, q);
                    s_mean[b] = q;
                }
            }
            vq[h] = (lc < r_rank) ? q * q : 0.0f;
        }
    }
#pragma unroll
    for (int h = 0; h < (BQ + 1) / 2; ++h) {
        float x = vq[h];
#pragma unroll
        for (int msk = 1; msk < 64; msk <<= 1) x += __shfl_xor(x, msk, 64);
        if (lane == 0 && (t >> 7) + 2 * h < BQ) s_bsum[w][h] = x;
    }
    __syncthreads();
    if (n_cb == 1) {  // the block is the whole GP (a Lanczos factor): finish here, no second hand-off
        if (t < B) {
            const int h = t >> 1, w0 = (t & 1) * 2;
            gp_gv_finish(m, B, i, t, 0.0f + (s_bsum[w0][h] + s_bsum[w0 + 1][h]), s_mean[t], os, nz, ys, mean_out,
                         std_out, cols, mean_cols, std_cols, hmean, hstd, BQ);
        }
        if (t == 0) atomicExch(&counters[(i * n_cb + cb) * kGvCtrStride], 0u);
        if constexpr (kSA) gp_sa_finish<BQ, SAM, SAK>(m, B, counters, *sa);
        return;
    }
    if (t < BQ) {  // query b = t: waves 0, 1 hold even b (slot b / 2), waves 2, 3 odd b
        const int h = t >> 1, w0 = (t & 1) * 2;
        st_sc1(blk + ((int64_t)i * n_cb + cb) * BQ + t, s_bsum[w0][h] + s_bsum[w0 + 1][h]);
    }
    // 7. arrival at GP i: the last of its blocks writes mean and std
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        atomicExch(&counters[(i * n_cb + cb) * kGvCtrStride], 0u);  // consumed: zero for the next call
        const unsigned tk = ticket(&counters[(m.n_s * n_cb + i) * kGvCtrStride]);
        if (tk >= (unsigned)n_cb) atomicOr(&counters[gp_fail_word(m)], 1u);
        s_last = tk == (unsigned)(n_cb - 1);
    }
    __syncthreads();
    if (!s_last) return;
    if (t < B)
        gp_gv_finish(m, B, i, t, sum_sc1(blk + (int64_t)i * n_cb * BQ + t, n_cb, BQ),
                     ld_sc1(meanraw + (int64_t)i * BQ + t), os, nz, ys, mean_out, std_out, cols, mean_cols, std_cols,
                     hmean, hstd, BQ);
    if (t == 0) atomicExch(&counters[(m.n_s * n_cb + i) * kGvCtrStride], 0u);
    if constexpr (kSA) gp_sa_finish<BQ, SAM, SAK>(m, B, counters, *sa);
}

template <int D, int BQ>
__global__ void __launch_bounds__(256) k_gp_gemv(rcbf_gp_model m, int64_t B, const float* __restrict__ xq,
                                                 int T, unsigned* counters, float* part, float* blk,
                                                 float* meanraw, float* __restrict__ mean_out,
                                                 float* __restrict__ std_out, GpCols cols,
                                                 float* __restrict__ mean_cols, float* __restrict__ std_cols) {
    gp_gemv_body<D, BQ>(m, B, xq, T, counters, part, blk, meanraw, mean_out, std_out, cols, mean_cols, std_cols,
                        nullptr);
}

// RCBF_SAC.get_safe_action(obs) with the fitted GP in ONE launch (rcbf_gp_obs_safe_action): the GEMV of
// the posterior on get_state(obs), then the last GP finisher solves the safe action (gp_sa_finish).
template <int D, int BQ, int SAM, int SAK>
__global__ void __launch_bounds__(256) k_gp_gemv_sa(rcbf_gp_model m, int64_t B, int T, unsigned* counters,
                                                    float* part, float* blk, float* meanraw,
                                                    float* __restrict__ mean_out, float* __restrict__ std_out,
                                                    GpSafeAction sa) {
    GpCols none{};
    gp_gemv_body<D, BQ, SAM, SAK>(m, B, nullptr, T, counters, part, blk, meanraw, mean_out, std_out, none, nullptr,
                                  nullptr, &sa);
}

// Split-K combine (the MFMA path, B > 8): one wave per (GP i, column block
// cb, query b) adds the n_split raw Q rows (fixed order) over the block's 128
// columns, then partial = sum_{col < r} Q^2 and meanraw = Q(b, r), as
// k_gp_qform's own epilogue.
// fin (one column block per GP, a Lanczos factor): the wave also finishes its
// query -- mean and std into the row and column outputs, the arithmetic of
// gp_mean_std -- so no finish launch follows.

__global__ void __launch_bounds__(256) k_gp_combine(rcbf_gp_model m, int64_t B, int n_cb, int n_split,
                                                    const float* __restrict__ qraw, float* __restrict__ partial,
                                                    float* __restrict__ meanraw, int fin, float* __restrict__ mean_out,
                                                    float* __restrict__ std_out, GpCols cols,
                                                    float* __restrict__ mean_cols, float* __restrict__ std_cols) {
    const int64_t wv = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wv >= (int64_t)m.n_s * n_cb * B) return;
    const int64_t b = wv % B;
    const int cb = (int)((wv / B) % n_cb);
    const int i = (int)(wv / (B * n_cb));
    const int64_t ldc = m.C_pad;
    float v = 0.0f, mq = 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int col = cb * kGpCols + 64 * h + lane;  // logical column: k_gp_qform stores Q by logical column
        // the n_split terms in order, 16 loads in flight at a time (a loop that adds each load as it
        // arrives pays a memory round trip per split: r05i, 11 splits ~ 9 us)
        const float* qp = qraw + ((int64_t)i * n_split * B + b) * ldc + col;
        const int64_t qs = B * ldc;
        float q = 0.0f;
        for (int s0 = 0; s0 < n_split; s0 += 16) {
            float a[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) a[u] = qp[(int64_t)min(s0 + u, n_split - 1) * qs];
#pragma unroll
            for (int u = 0; u < 16; ++u) q += (s0 + u < n_split) ? a[u] : 0.0f;
        }
        v += (col < m.r) ? q * q : 0.0f;
        if (col == m.r) {
            meanraw[(int64_t)i * B + b] = q;
            mq = q;
        }
    }
#pragma unroll
    for (int msk = 1; msk < 64; msk <<= 1) v += __shfl_xor(v, msk, 64);
    if (fin) {  // n_cb == 1: this wave saw every column of GP i at query b
#pragma unroll
        for (int msk = 1; msk < 64; msk <<= 1) mq += __shfl_xor(mq, msk, 64);  // the one lane holding column r
        if (lane == 0)
            gp_gv_finish(m, B, i, (int)b, 0.0f + v, mq, m.outscale[i], m.noise[i], m.y_scale[i], mean_out, std_out,
                         cols, mean_cols, std_cols);
        return;
    }
    if (lane == 0) partial[((int64_t)i * n_cb + cb) * B + b] = v;
}

// mean/std (B, n_s) row-major like predict_disturbance's (n_test, n_s) output;
// GpCols: the output dimensions written in column layout (rcbf_gp_predict_cols).

// mean and std of GP i at query b (dynamics.py:371-380 after gpytorch)
__device__ __forceinline__ void gp_mean_std(const rcbf_gp_model& m, int64_t B, int n_cb, const float* partial,
                                            const float* meanraw, int i, int64_t b, float& mu, float& sd) {
    float q = 0.0f;  // the n_cb block sums in order, 16 loads in flight at a time
    const float* pp = partial + (int64_t)i * n_cb * B + b;
    for (int c0 = 0; c0 < n_cb; c0 += 16) {
        float a[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) a[u] = pp[(int64_t)min(c0 + u, n_cb - 1) * B];
#pragma unroll
        for (int u = 0; u < 16; ++u) q += (c0 + u < n_cb) ? a[u] : 0.0f;
    }
    const float lat = fmaxf(m.outscale[i] - q, 0.0f);  // latent posterior variance
    const float var = lat + m.noise[i];                  // likelihood(model(x)).variance
    mu = meanraw[(int64_t)i * B + b] * m.y_scale[i];
    sd = sqrtf(var) * m.y_scale[i];
}

// (B, n_s) row outputs, thread e = b n_s + i
__global__ void __launch_bounds__(256) k_gp_finish(rcbf_gp_model m, int64_t B, int n_cb,
                                                   const float* __restrict__ partial,
                                                   const float* __restrict__ meanraw, float* __restrict__ mean_out,
                                                   float* __restrict__ std_out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= B * m.n_s) return;
    float mu, sd;
    gp_mean_std(m, B, n_cb, partial, meanraw, (int)(e % m.n_s), e / m.n_s, mu, sd);
    if (mean_out) mean_out[e] = mu;
    if (std_out) std_out[e] = sd;
}

// column outputs (cols.n, B), thread e = c B + b: consecutive lanes store
// consecutive b of one column (the same arithmetic as k_gp_finish, so the
// same values bit for bit)
__global__ void __launch_bounds__(256) k_gp_finish_cols(rcbf_gp_model m, int64_t B, int n_cb,
                                                        const float* __restrict__ partial,
                                                        const float* __restrict__ meanraw, GpCols cols,
                                                        float* __restrict__ mean_cols, float* __restrict__ std_cols) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= B * cols.n) return;
    const int c = (int)(e / B);
    float mu, sd;
    gp_mean_std(m, B, n_cb, partial, meanraw, cols.idx[c], e % B, mu, sd);
    if (mean_cols) mean_cols[e] = mu;
    if (std_cols) std_cols[e] = sd;
}

// Split-K factor: 1 when the (query tile x column block x GP) grid already
// gives every CU several workgroups; otherwise enough splits of the training
// rows for ~6 workgroups per CU (3 resident per CU at 160 VGPRs), capped at one
// split per 256-row LDS chunk, the last chunk counted even when partial: rank
// 100 at N = 3 000, B = 256 then runs 12 splits of 256 rows (240 workgroups,
// 8 blocks of 32 rows each) instead of 11 of 288 (9 blocks): 39.2 -> 36.4 us
// (profiles/r06/gp_split_sweep_r06t.txt).
constexpr int kGvMaxB = 8;  // B <= 8: the streaming GEMV path

int gp_split(const rcbf_gp_model* m, int64_t B) {
    if (B <= kGvMaxB) return 1;  // the GEMV path tiles the rows itself
#ifdef RCBF_STUDY_GP_SPLIT  // study builds only: the split count from the environment
    if (const char* e = getenv("RCBF_GP_SPLIT")) return atoi(e) < 1 ? 1 : atoi(e);
#endif
    const int64_t cus = num_cus();
    const int64_t tiles = ((B + kGpRows - 1) / kGpRows) * (m->C_pad / kGpCols) * m->n_s;
    const int64_t want = 6LL * cus;
    if (tiles >= want / 2) return 1;
    int64_t sk = (want + tiles - 1) / tiles;
    const int64_t cap = (m->N_pad + kGpChunk - 1) / kGpChunk;
    sk = sk < cap ? sk : cap;
    return sk < 1 ? 1 : (int)sk;
}

}  // namespace

extern "C" {

int64_t rcbf_gp_workspace_floats(const rcbf_gp_model* m, int64_t B) {
    if (!m || B < 0 || m->C_pad < kGpCols || m->n_s < 1) return -1;
    const int64_t n_cb = m->C_pad / kGpCols;
    const int64_t cw = gp_counter_words(*m);
    if (B <= kGvMaxB)  // GEMV: tile partials (32 columns x 8 queries), block sums, mean column, the fused
                       // safe action's mean / std hand-off
        return cw + (int64_t)m->n_s * gp_gv_tiles(*m) * kGvMaxB * kGpCols + (int64_t)m->n_s * (n_cb + 3) * kGvMaxB;
    const int sk = gp_split(m, B);
    // partials for up to 2 launches per block, + means, + the split-K raw Q tiles
    return cw + (int64_t)m->n_s * (2 * n_cb + 1) * B + (sk > 1 ? (int64_t)sk * m->n_s * B * m->C_pad : 0);
}

int rcbf_gp_workspace_init(const rcbf_gp_model* m, float* workspace, hipStream_t stream) {
    if (!m || !workspace) return RCBF_E_NULL;
    if (m->C_pad < kGpCols || m->n_s < 1) return RCBF_E_BAD_SHAPE;
    return (int)hipMemsetAsync(workspace, 0, (size_t)gp_counter_words(*m) * 4, stream);
}

int rcbf_gp_workspace_check(const rcbf_gp_model* m, float* workspace, hipStream_t stream) {
    if (!m || !workspace) return RCBF_E_NULL;
    if (m->C_pad < kGpCols || m->n_s < 1) return RCBF_E_BAD_SHAPE;
    // every counter word and the fail word: once the stream has drained, a clean workspace reads all zero.  A
    // set fail word is a call that drew a ticket past its counter's arrival count; a non-zero counter is a
    // call whose counter started off by less than that (an early arrival took the "last" ticket, reset the
    // counter, and the late ones left it non-zero without ever drawing a ticket past the count)
    std::vector<unsigned> h((size_t)gp_counter_words(*m));
    int rc = (int)hipMemcpyAsync(h.data(), workspace, h.size() * 4, hipMemcpyDeviceToHost, stream);
    if (!rc) rc = (int)hipStreamSynchronize(stream);
    if (rc) return rc;
    bool bad = false;
    for (unsigned v : h) bad |= v != 0;
    if (!bad) return 0;
    // zero every counter and the fail word, so the next call is clean
    rc = rcbf_gp_workspace_init(m, workspace, stream);
    if (!rc) rc = (int)hipStreamSynchronize(stream);
    return rc ? rc : RCBF_E_GP_HANDOFF;
}

int rcbf_gp_predict(const rcbf_gp_model* m, int64_t B, const float* x, float* mean_out, float* std_out,
                    float* workspace, hipStream_t stream) {
    if (!mean_out || !std_out) return RCBF_E_NULL;
    return rcbf_gp_predict_cols(m, B, x, mean_out, std_out, nullptr, 0, nullptr, nullptr, workspace, stream);
}

int rcbf_gp_predict_cols(const rcbf_gp_model* m, int64_t B, const float* x, float* mean_out, float* std_out,
                         const int32_t* cols, int32_t n_cols, float* mean_cols, float* std_cols, float* workspace,
                         hipStream_t stream) {
    if (!m) return RCBF_E_NULL;
    GpCols gc{};
    if (n_cols < 0 || n_cols > 10 || (n_cols > 0 && !cols)) return RCBF_E_BAD_SHAPE;
    gc.n = (mean_cols || std_cols) ? n_cols : 0;
    for (int c = 0; c < gc.n; ++c) {
        if (cols[c] < 0 || cols[c] >= m->n_s) return RCBF_E_BAD_SHAPE;
        gc.idx[c] = cols[c];
    }
    if (!mean_out && !std_out && gc.n == 0) return RCBF_E_NULL;  // nothing to write
    if (B < 0 || m->n_s < 1 || m->n_s > 10 || m->N < 1 || m->N_pad % 32 || m->N_pad < m->N || m->r < 1 ||
        m->r > m->N || m->C_pad % kGpCols || m->C_pad < m->r + 1)
        return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !workspace || !m->xt || !m->tn2 || !m->Rt || !m->x_std || !m->inv_sl ||
        !m->outscale || !m->noise || !m->y_scale)
        return RCBF_E_NULL;
    const int n_cb = m->C_pad / kGpCols;
    // the arrival counters of the GEMV path sit first (zero-filled by the caller once -- torch.zeros or
    // rcbf_gp_workspace_init -- and left zero by every call; a call that finds one non-zero sets the fail
    // word rcbf_gp_workspace_check reads)
    unsigned* counters = reinterpret_cast<unsigned*>(workspace);
    float* ws = workspace + gp_counter_words(*m);
    if (B <= kGvMaxB) {
        const int T = gp_gv_tiles(*m);
        float* part = ws;
        float* blk = part + (int64_t)m->n_s * T * kGvMaxB * kGpCols;
        float* mraw = blk + (int64_t)m->n_s * n_cb * kGvMaxB;
        dim3 gv((unsigned)T, (unsigned)m->n_s);
#define RCBF_GV_L(DD, BB)                                                                                  \
    hipLaunchKernelGGL((k_gp_gemv<DD, BB>), gv, dim3(256), 0, stream, *m, B, x, T, counters, part, blk, mraw, \
                       mean_out, std_out, gc, mean_cols, std_cols)
#define RCBF_GV_B(DD)           \
    do {                        \
        if (B == 1)             \
            RCBF_GV_L(DD, 1);   \
        else if (B == 2)        \
            RCBF_GV_L(DD, 2);   \
        else if (B <= 4)        \
            RCBF_GV_L(DD, 4);   \
        else                    \
            RCBF_GV_L(DD, 8);   \
    } while (0)
        switch (m->n_s) {
            case 3:
                RCBF_GV_B(3);
                break;
            case 10:
                RCBF_GV_B(10);
                break;
            default:
                return RCBF_E_BAD_SHAPE;
        }
#undef RCBF_GV_B
#undef RCBF_GV_L
        return launch_status();
    }
    // CT = 2 (half-width column tiles, twice the workgroups) measured no faster
    // at B = 256 (profiles/r01/gp_predict_roofline.jsonl), so every batch uses CT = 4
    const int n_part = n_cb;
    float* partial = ws;
    float* meanraw = ws + (int64_t)m->n_s * 2 * n_cb * B;
    const int sk = gp_split(m, B);
    float* qraw = meanraw + (int64_t)m->n_s * B;
    {
        dim3 g((unsigned)((B + kGpRows - 1) / kGpRows), (unsigned)n_part, (unsigned)(m->n_s * sk));
#define RCBF_GP_L(DD)                                                                                           \
    do {                                                                                                        \
        if (sk > 1 && kGpSk2)                                                                                   \
            hipLaunchKernelGGL((k_gp_qform_sk2<DD>), g, dim3(512), 0, stream, *m, B, x, partial, meanraw, sk,   \
                               qraw);                                                                           \
        else if (sk > 1)                                                                                        \
            hipLaunchKernelGGL((k_gp_qform<DD, 4, true>), g, dim3(256), 0, stream, *m, B, x, partial, meanraw, \
                               sk, qraw);                                                                       \
        else                                                                                                    \
            hipLaunchKernelGGL((k_gp_qform<DD, 4>), g, dim3(256), 0, stream, *m, B, x, partial, meanraw, 1,    \
                               nullptr);                                                                        \
    } while (0)
        switch (m->n_s) {  // D = n_s: the GP inputs are the full state
            case 3:
                RCBF_GP_L(3);
                break;
            case 10:
                RCBF_GP_L(10);
                break;
            default:
                return RCBF_E_BAD_SHAPE;
        }
#undef RCBF_GP_L
    }
    if (sk > 1) {
        const int64_t waves = (int64_t)m->n_s * n_cb * B;
        const int fin = n_cb == 1;  // a Lanczos factor: the combine also finishes (no k_gp_finish launch)
        hipLaunchKernelGGL(k_gp_combine, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, stream, *m, B, n_cb, sk,
                           qraw, partial, meanraw, fin, mean_out, std_out, gc, mean_cols, std_cols);
        if (fin) return launch_status();
    }
    if (mean_out || std_out) {
        const int64_t tot = B * m->n_s;
        hipLaunchKernelGGL(k_gp_finish, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, *m, B, n_part,
                           partial, meanraw, mean_out, std_out);
    }
    if (gc.n > 0) {
        const int64_t tot = B * gc.n;
        hipLaunchKernelGGL(k_gp_finish_cols, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, *m, B,
                           n_part, partial, meanraw, gc, mean_cols, std_cols);
    }
    return launch_status();
}


int rcbf_gp_obs_safe_action(const rcbf_params* prm, const rcbf_gp_model* m, int64_t B, const float* obs,
                            const float* u_rl, float* mean_out, float* std_out, float* u_out, float* u_host,
                            uint32_t* done_word, uint32_t seq, int32_t* status_out, int32_t* fail_flag,
                            float* workspace, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (!m) return RCBF_E_NULL;
    if (B != 1) return RCBF_E_BAD_SHAPE;  // the per-env-step query (main.py:93); batches take rcbf_gp_predict
    if (m->n_s < 1 || m->n_s > 10 || m->N < 1 || m->N_pad % 32 || m->N_pad < m->N || m->r < 1 || m->r > m->N ||
        m->C_pad % kGpCols || m->C_pad < m->r + 1)
        return RCBF_E_BAD_SHAPE;
    const bool cars = prm->mode == RCBF_MODE_SIMULATED_CARS;
    if (m->n_s != (cars ? 10 : 3)) return RCBF_E_BAD_SHAPE;  // one GP per state dimension of the env
    if (prm->solver != RCBF_SOLVER_ACTIVE_SET) return RCBF_E_BAD_MODE;
    if (!obs || !u_rl || !workspace || !m->xt || !m->tn2 || !m->Rt || !m->x_std || !m->inv_sl || !m->outscale ||
        !m->noise || !m->y_scale)
        return RCBF_E_NULL;
    if (!u_out && !u_host) return RCBF_E_NULL;  // nowhere to put the action
    const int n_cb = m->C_pad / kGpCols;
    const int T = gp_gv_tiles(*m);
    unsigned* counters = reinterpret_cast<unsigned*>(workspace);
    float* part = workspace + gp_counter_words(*m);
    float* blk = part + (int64_t)m->n_s * T * kGvMaxB * kGpCols;
    float* mraw = blk + (int64_t)m->n_s * n_cb * kGvMaxB;
    GpSafeAction sa{};
    sa.prm = *prm;
    sa.obs = obs;
    sa.u_rl = u_rl;
    sa.hmean = mraw + (int64_t)m->n_s * kGvMaxB;
    sa.hstd = sa.hmean + (int64_t)m->n_s * kGvMaxB;
    sa.u_out = u_out;
    sa.u_host = u_host;
    sa.done_word = done_word;
    sa.status_out = status_out;
    sa.fail_flag = fail_flag;
    sa.seq = seq;
    dim3 gv((unsigned)T, (unsigned)m->n_s);
#define RCBF_GVSA_L(DD, MODE_, K_)                                                                            \
    hipLaunchKernelGGL((k_gp_gemv_sa<DD, 1, MODE_, K_>), gv, dim3(256), 0, stream, *m, B, T, counters, part, blk, \
                       mraw, mean_out, std_out, sa)
    if (cars) {
        RCBF_GVSA_L(10, RCBF_MODE_SIMULATED_CARS, 1);
    } else {
        switch (prm->num_hazards) {
            case 1: RCBF_GVSA_L(3, RCBF_MODE_UNICYCLE, 1); break;
            case 2: RCBF_GVSA_L(3, RCBF_MODE_UNICYCLE, 2); break;
            case 3: RCBF_GVSA_L(3, RCBF_MODE_UNICYCLE, 3); break;
            case 4: RCBF_GVSA_L(3, RCBF_MODE_UNICYCLE, 4); break;
            case 5: RCBF_GVSA_L(3, RCBF_MODE_UNICYCLE, 5); break;
            case 6: RCBF_GVSA_L(3, RCBF_MODE_UNICYCLE, 6); break;
            case 7: RCBF_GVSA_L(3, RCBF_MODE_UNICYCLE, 7); break;
            case 8: RCBF_GVSA_L(3, RCBF_MODE_UNICYCLE, 8); break;
            default: return RCBF_E_BAD_SHAPE;
        }
    }
#undef RCBF_GVSA_L
    if (int rc = launch_status()) return rc;
    if (!done_word) return 0;
    // the result is on the host once the word reads `seq` (the kernel's last stage publishes it system-wide);
    // every 4096 polls ask the stream, so a failed kernel returns its error instead of spinning.  A kernel
    // that completed without publishing never reached its last stage: a hand-off counter was not zero at
    // the start (the fail word is set; rcbf_gp_workspace_check reports and repairs it)
    volatile uint32_t* w = done_word;
    for (uint32_t n = 1;; ++n) {
        if (*w == seq) return 0;
        __builtin_ia32_pause();
        if ((n & 4095) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) return *w == seq ? 0 : RCBF_E_GP_HANDOFF;
            if (q != hipErrorNotReady) return (int)q;
        }
    }
}

}  // extern "C"
