// rcbf_wave_qp.hip -- STUDY build (not in librcbf_hip.so): the north star's
// "one QP per wavefront" interior point, to measure it against the product's
// one-QP-per-lane solvers (the qpth call it would replace is
// rcbf_sac/diff_cbf_qp.py:107,139).
//
// The same primal-dual interior-point algorithm as pdipm_solve
// (rcbf_device.hpp: qpth's initial point, Mehrotra predictor-corrector, 0.999
// step to the boundary, best-iterate tracking, notImprovedLim = 10) with the
// rows spread over the lanes: W lanes per QP (W = 64: one QP per wavefront;
// W = 16: four QPs per wavefront), lane r of a group holds row r (G_r, h_r,
// s_r, lam_r), and every sum or min over rows -- the dual residual G' lam,
// s'lam, the normal matrix G' D G and its right-hand sides, the step lengths
// -- is a butterfly reduction over the group's lanes (__shfl_xor).  The
// n x n solve is repeated in every lane.  Diagonal P, fp32 rows, fp64
// arithmetic, rows optionally normalised like CBFQPLayer.solve_qp.
//
// Built by scripts/wave_qp_study.py --build into build/study/librcbf_wave_qp.so.
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

template <int W>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
    for (int o = W / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int W>
__device__ __forceinline__ double group_min(double v) {
#pragma unroll
    for (int o = W / 2; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}

template <int N>
__device__ __forceinline__ void solve_sym(const double H[N][N], const double* b, double* x) {
    double S[N][N];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) S[i][j] = H[i][j];
    ldl_solve<N>(S, b, x);
}

template <int N, int W>
__global__ void __launch_bounds__(256) k_wave_pdipm(int64_t B, int m, const float* __restrict__ P,
                                                    const float* __restrict__ G, const float* __restrict__ h,
                                                    int normalize, int max_iter, double eps,
                                                    float* __restrict__ z_out, int32_t* __restrict__ iters_out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t qp = t / W;
    const int r = (int)(t % W);
    const bool valid_qp = qp < B;
    const bool row = valid_qp && r < m;
    double g[N], hr = 0.0, p[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        g[k] = row ? (double)G[(qp * m + r) * N + k] : 0.0;
        p[k] = valid_qp ? (double)P[qp * N * N + k * N + k] : 1.0;
    }
    hr = row ? (double)h[qp * m + r] : 0.0;
    if (normalize && row) {  // diff_cbf_qp.py:103-106 on this lane's row
        float mx = fabsf((float)hr);
#pragma unroll
        for (int k = 0; k < N; ++k) mx = fmaxf(mx, fabsf((float)g[k]));
#pragma unroll
        for (int k = 0; k < N; ++k) g[k] = (double)((float)g[k] / mx);
        hr = (double)((float)hr / mx);
    }
    // initial point (qpth): (P + G'G) x = G'h, s = h - Gx, lam = Gx - h, shifted positive
    double x[N];
    {
        double H[N][N], rhs[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
#pragma unroll
            for (int j = 0; j <= i; ++j) {
                const double v = group_sum<W>(g[i] * g[j]) + (i == j ? p[i] : 0.0);
                H[i][j] = v;
                H[j][i] = v;
            }
            rhs[i] = group_sum<W>(g[i] * hr);
        }
        solve_sym<N>(H, rhs, x);
    }
    double gx = dotd<N>(g, x);
    double s = hr - gx, lam = gx - hr;
    const double smin = group_min<W>(row ? s : kInf), lmin = group_min<W>(row ? lam : kInf);
    if (smin < 0.0) s -= smin - 1.0;
    if (lmin < 0.0) lam -= lmin - 1.0;
    if (!row) {
        s = 1.0;
        lam = 0.0;
    }
    double best = kInf, bx[N];
#pragma unroll
    for (int k = 0; k < N; ++k) bx[k] = x[k];
    int not_improved = 0, it = 0, qit = max_iter;  // qit: this QP's iterations
    bool done = !valid_qp;
    const double fm = (double)m;
    for (; it < max_iter; ++it) {
        if (__ballot(!done) == 0) break;
        // residuals: rx = P x + G' lam, rz = G x + s - h, mu = s'lam / m
        double rx[N];
#pragma unroll
        for (int k = 0; k < N; ++k) rx[k] = p[k] * x[k] + group_sum<W>(g[k] * lam);
        const double rz = row ? dotd<N>(g, x) + s - hr : 0.0;
        const double sz = group_sum<W>(row ? s * lam : 0.0);
        const double zr = group_sum<W>(rz * rz);
        const double mu = fabs(sz / fm);
        const double res = sqrt(zr) + sqrt(dotd<N>(rx, rx)) + fm * mu;
        if (!done) {
            if (res < best) {
                best = res;
                not_improved = 0;
#pragma unroll
                for (int k = 0; k < N; ++k) bx[k] = x[k];
            } else {
                ++not_improved;
            }
            if (best < eps || not_improved >= 10) {
                done = true;
                qit = it;
            }
        }
        if (__ballot(!done) == 0) break;
        // normal matrix H = P + G' D G, D = lam / s
        const double d = row ? lam * rcp64(s) : 0.0;
        double H[N][N];
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) {
                const double v = group_sum<W>(g[i] * d * g[j]) + (i == j ? p[i] : 0.0);
                H[i][j] = v;
                H[j][i] = v;
            }
        auto kkt = [&](double rs, const double* rxv, double rzv, double* dx, double& ds, double& dl) {
            double rhs[N];
#pragma unroll
            for (int k = 0; k < N; ++k) rhs[k] = -rxv[k] + group_sum<W>(row ? g[k] * (rs - d * rzv) : 0.0);
            solve_sym<N>(H, rhs, dx);
            ds = row ? -rzv - dotd<N>(g, dx) : 0.0;
            dl = row ? -rs - d * ds : 0.0;
        };
        double dx[N], ds, dl;
        kkt(lam, rx, rz, dx, ds, dl);  // affine direction
        double a = kInf;
        if (row && dl < 0.0) a = fmin(a, -lam * rcp64(dl));
        if (row && ds < 0.0) a = fmin(a, -s * rcp64(ds));
        const double a_aff = fmin(1.0, group_min<W>(a));
        const double t3 = group_sum<W>(row ? (s + a_aff * ds) * (lam + a_aff * dl) : 0.0);
        double sig = t3 * rcp64(sz);
        sig = sig * sig * sig;
        double dxc[N], dsc, dlc;
        const double zero[N] = {};
        kkt(row ? (-mu * sig + ds * dl) * rcp64(s) : 0.0, zero, 0.0, dxc, dsc, dlc);  // corrector
#pragma unroll
        for (int k = 0; k < N; ++k) dx[k] += dxc[k];
        ds += dsc;
        dl += dlc;
        a = kInf;
        if (row && dl < 0.0) a = fmin(a, -lam * rcp64(dl));
        if (row && ds < 0.0) a = fmin(a, -s * rcp64(ds));
        double amax = group_min<W>(a);
        if (amax == kInf) amax = 1.0;
        const double alpha = done ? 0.0 : fmin(1.0, 0.999 * amax);
#pragma unroll
        for (int k = 0; k < N; ++k) x[k] += alpha * dx[k];
        if (row) {
            s += alpha * ds;
            lam += alpha * dl;
        }
    }
    if (valid_qp && r == 0) {
#pragma unroll
        for (int k = 0; k < N; ++k) z_out[qp * N + k] = (float)bx[k];
        if (iters_out) iters_out[qp] = qit;
    }
}

}  // namespace

extern "C" {

// z_out (B, n) fp32 (best iterate, no polish); iters_out [nullable] (B,) i32 per QP;
// lanes_per_qp 64 (one QP per wavefront) or 16.
int rcbf_study_wave_pdipm(int64_t B, int32_t n, int32_t m, const float* P, const float* G, const float* h,
                          int32_t normalize, int32_t max_iter, double eps, int32_t lanes_per_qp, float* z_out,
                          int32_t* iters_out, hipStream_t stream) {
    if (B <= 0) return 0;
    if (n < 2 || n > 3 || m < 1 || m > lanes_per_qp || (lanes_per_qp != 64 && lanes_per_qp != 16))
        return RCBF_E_BAD_SHAPE;
    if (!P || !G || !h || !z_out) return RCBF_E_NULL;
    const int64_t threads = B * lanes_per_qp;
    dim3 g((unsigned)((threads + 255) / 256)), b(256);
#define RCBF_WQ(NN, WW)                                                                                         \
    hipLaunchKernelGGL((k_wave_pdipm<NN, WW>), g, b, 0, stream, B, m, P, G, h, normalize, max_iter, eps, z_out, \
                       iters_out)
    if (n == 2 && lanes_per_qp == 64)
        RCBF_WQ(2, 64);
    else if (n == 2)
        RCBF_WQ(2, 16);
    else if (lanes_per_qp == 64)
        RCBF_WQ(3, 64);
    else
        RCBF_WQ(3, 16);
#undef RCBF_WQ
    return (int)hipGetLastError();
}

}  // extern "C"
