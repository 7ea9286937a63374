// rcbf_qp_common.hpp -- the generic QP machinery shared by the QP
// translation units (rcbf_qp.hip: fp32 forward, rcbf_qp_f64.hip: fp64
// forward, rcbf_qp_bwd.hip: backward): LDS staging of the AoS per-QP
// tensors, the structured fast path, the forward kernel k_qp_solve and its
// launcher.  Split over several TUs so they compile in parallel.
#pragma once

#include "rcbf_common.hpp"

namespace rcbf_qp {

using namespace rcbf;


// ---------------------------------------------------------------------------
// Generic QP kernels (CBFQPLayer.solve_qp / cbf_layer and their autograd,
// diff_cbf_qp.py:81-144; CascadeCBFLayer.solve_qp, cbf_qp.py:242-286).
// One QP per lane.  The per-QP tensors are AoS rows -- G (B, m, n), h (B, m),
// P (B, n, n), q (B, n) -- so a workgroup's QPs are one contiguous chunk of
// each tensor: the workgroup stages its chunks into LDS with coalesced loads
// (consecutive lanes read consecutive words), and each lane then reads its own
// rows from LDS at an odd word stride (no bank conflicts).  The backward's
// gradient rows go out the same way.
// ---------------------------------------------------------------------------
constexpr int kQPBlock = 128;

__host__ __device__ inline int odd_stride(int w) { return w | 1; }

// LDS <- the workgroup's chunk of an AoS tensor with W <= MAXW elements per
// QP, at row stride odd_stride(W) words in LDS: every lane first issues all of
// its (coalesced, predicated) loads, then writes them to LDS, so the loads are
// in flight together.  fp32 chunks that start 16-B aligned move as float4:
// for odd W the padded layout IS the linear one (one ds_write_b128 per
// float4); for even W each element lands at e + e / W (the row's pad word).
template <typename T, int MAXW>
__device__ __forceinline__ void stage_in(const T* __restrict__ src, T* lds, int nb, int W) {
    const int Wp = odd_stride(W), tot = nb * W;
    if constexpr (sizeof(T) == 4) {
        if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            constexpr int J4 = (MAXW + 3) / 4;  // float4s per lane at a full chunk
            const int n4 = tot >> 2;
            typedef float f4 __attribute__((ext_vector_type(4)));
            f4 v[J4];
#pragma unroll
            for (int j = 0; j < J4; ++j) {
                const int c4 = threadIdx.x + j * kQPBlock;
                v[j] = c4 < n4 ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(src) + c4) : f4{0, 0, 0, 0};
            }
            const int rem = tot - 4 * n4;  // < 4 trailing words
            const T tail = threadIdx.x < rem ? ld_in(src + 4 * n4 + threadIdx.x) : T(0);
            if (W & 1) {
#pragma unroll
                for (int j = 0; j < J4; ++j) {
                    const int c4 = threadIdx.x + j * kQPBlock;
                    if (c4 < n4) *reinterpret_cast<f4*>(lds + 4 * c4) = v[j];
                }
                if (threadIdx.x < rem) lds[4 * n4 + threadIdx.x] = tail;
            } else {
                const float invW = 1.0f / (float)W;  // e / W exact below 2^16 (e + 0.5 keeps off the integers)
                auto put = [&](int e, T x) { lds[e + (int)(((float)e + 0.5f) * invW)] = x; };
#pragma unroll
                for (int j = 0; j < J4; ++j) {
                    const int c4 = threadIdx.x + j * kQPBlock;
                    if (c4 < n4) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) put(4 * c4 + t, v[j][t]);
                    }
                }
                if (threadIdx.x < rem) put(4 * n4 + threadIdx.x, tail);
            }
            return;
        }
    }
    const int e0 = threadIdx.x, q0 = e0 / W, c0 = e0 - q0 * W;
    const int dq = kQPBlock / W, dc = kQPBlock - dq * W;
    T v[MAXW];
#pragma unroll
    for (int j = 0; j < MAXW; ++j) {
        const int e = e0 + j * kQPBlock;
        v[j] = e < tot ? ld_in(src + e) : T(0);
    }
    int q = q0, c = c0;
#pragma unroll
    for (int j = 0; j < MAXW; ++j) {
        if (e0 + j * kQPBlock < tot) lds[q * Wp + c] = v[j];
        q += dq;
        c += dc;
        if (c >= W) {
            c -= W;
            ++q;
        }
    }
}

// the workgroup's chunk of an AoS output tensor <- LDS (the same two forms)
template <typename T>
__device__ __forceinline__ void stage_out(T* __restrict__ dst, const T* lds, int nb, int W) {
    const int Wp = odd_stride(W), tot = nb * W;
    if constexpr (sizeof(T) == 4) {
        if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            const int n4 = tot >> 2, rem = tot - 4 * n4;
            const float invW = 1.0f / (float)W;
            auto get = [&](int e) { return (W & 1) ? lds[e] : lds[e + (int)(((float)e + 0.5f) * invW)]; };
            for (int c4 = threadIdx.x; c4 < n4; c4 += kQPBlock) {
                f4 v;
                if (W & 1) {
                    v = *reinterpret_cast<const f4*>(lds + 4 * c4);
                } else {
#pragma unroll
                    for (int t = 0; t < 4; ++t) v[t] = get(4 * c4 + t);
                }
                __builtin_nontemporal_store(v, reinterpret_cast<f4*>(dst) + c4);
            }
            if (threadIdx.x < rem) dst[4 * n4 + threadIdx.x] = get(4 * n4 + threadIdx.x);
            return;
        }
    }
    int e = threadIdx.x, q = e / W, c = e - q * W;
    const int dq = kQPBlock / W, dc = kQPBlock - dq * W;
    for (; e < tot; e += kQPBlock) {
        dst[e] = lds[q * Wp + c];
        q += dq;
        c += dc;
        if (c >= W) {
            c -= W;
            ++q;
        }
    }
}

// LDS words of one workgroup's staged QP inputs (G, h, P, q)
__host__ __device__ inline int qp_lds_words(int n, int m) {
    return kQPBlock * (odd_stride(m * n) + odd_stride(m) + odd_stride(n * n) + odd_stride(n));
}

template <int N, int MP, typename T>
struct StagedQP {
    T G[MP][N], h[MP];
    double P[N][N], q[N];
    bool diag, qzero;
};

template <int N, int MP, typename T>
__device__ __forceinline__ void staged_read(const T* sG, const T* sh, const T* sP, const T* sq, int lane, int m,
                                            bool has_q, StagedQP<N, MP, T>& Q) {
    const int wg = odd_stride(m * N), wh = odd_stride(m), wp = odd_stride(N * N), wq = odd_stride(N);
#pragma unroll
    for (int r = 0; r < MP; ++r) {
        const bool in = r < m;
#pragma unroll
        for (int k = 0; k < N; ++k) Q.G[r][k] = in ? sG[lane * wg + r * N + k] : T(0);
        Q.h[r] = in ? sh[lane * wh + r] : T(1);  // padding rows: 0 z <= 1, never active
    }
    Q.diag = true;
    Q.qzero = true;
#pragma unroll
    for (int a = 0; a < N; ++a) {
        Q.q[a] = has_q ? (double)sq[lane * wq + a] : 0.0;
        Q.qzero = Q.qzero && Q.q[a] == 0.0;
#pragma unroll
        for (int b = 0; b < N; ++b) {
            Q.P[a][b] = (double)sP[lane * wp + a * N + b];
            if (a != b) Q.diag = Q.diag && Q.P[a][b] == 0.0;
        }
    }
}

// Is this QP the CBF layer's structure, for which the exact closed-form
// solvers apply?  (diagonal P, q = 0; n = 2, m = 4: the cars rows -- slack
// column < 0 on the two CBF rows, actuator rows [+, 0], [-, 0]; n = 3,
// m = K + 4: the unicycle rows -- slack column < 0 on K hazard rows, then the
// box [+,0,0], [-,0,0], [0,+,0], [0,-,0].)
template <int N, int MP, typename T>
__device__ __forceinline__ bool layer_structured(const StagedQP<N, MP, T>& Q, int m) {
    if (!(Q.diag && Q.qzero)) return false;
    if constexpr (N == 2) {
        if (m != 4 || MP < 4) return false;
        return Q.G[0][1] < T(0) && Q.G[1][1] < T(0) && Q.G[2][0] > T(0) && Q.G[2][1] == T(0) &&
               Q.G[3][0] < T(0) && Q.G[3][1] == T(0);
    } else if constexpr (N == 3) {
        const int K = m - 4;
        if (K < 1 || K > RCBF_MAX_HAZARDS || K + 4 > MP) return false;
        bool ok = true;
#pragma unroll
        for (int r = 0; r < MP; ++r) {
            const bool cbf = r < K;
            const int b = r - K;  // box row 0..3
            const bool box = !cbf && b < 4;
            const int c = b >> 1;      // bounded coordinate
            const bool up = (b & 1) == 0;
            const T g0 = Q.G[r][0], g1 = Q.G[r][1], g2 = Q.G[r][2];
            const bool box_ok = (c == 0 ? (up ? g0 > T(0) : g0 < T(0)) && g1 == T(0)
                                        : (up ? g1 > T(0) : g1 < T(0)) && g0 == T(0)) &&
                                g2 == T(0);
            ok = ok && (cbf ? g2 < T(0) : (box ? box_ok : true));
        }
        return ok;
    } else {
        return false;
    }
}

template <int N, int MP, typename T>
__device__ __forceinline__ void structured_solve(const StagedQP<N, MP, T>& Q, int m, double* z, int& status) {
    PMat<N, true> pm;
    double pd[N];
#pragma unroll
    for (int k = 0; k < N; ++k) pd[k] = Q.P[k][k];
    pmat_set_diag_rt<N>(pm, pd);
    if constexpr (N == 2 && MP >= 4) {
        cars_qp_1d<T>(pm, Q.G, Q.h, z, status);
    } else if constexpr (N == 3) {
        switch (m - 4) {
#define RCBF_UNI_CASE(KK)                                                   \
    case KK:                                                                \
        if constexpr (KK + 4 <= MP) uni_qp_2d<KK, T>(pm, Q.G, Q.h, z, status); \
        break;
            RCBF_UNI_CASE(1)
            RCBF_UNI_CASE(2)
            RCBF_UNI_CASE(3)
            RCBF_UNI_CASE(4)
            RCBF_UNI_CASE(5)
            RCBF_UNI_CASE(6)
            RCBF_UNI_CASE(7)
            RCBF_UNI_CASE(8)
#undef RCBF_UNI_CASE
            default:
                break;
        }
    }
}

// Full SPD P = L L' (Cholesky): in y = L' z the QP has P = I, rows G L^-T
// and linear term L^-1 q, so the Goldfarb-Idnani steps use the cheap
// identity-P algebra; z = L^-T y, and the multipliers / active set are those
// of the original QP.  Returns false (and leaves res alone) if P is not SPD.
template <int N, int MP, typename T>
__device__ __forceinline__ bool gi_solve_chol(const StagedQP<N, MP, T>& Q, int max_iter, QPResult<N, MP>& res) {
    double L[N][N], id[N];
    bool spd = true;
#pragma unroll
    for (int a = 0; a < N; ++a) {
#pragma unroll
        for (int b = 0; b <= a; ++b) {
            double acc = Q.P[a][b];
#pragma unroll
            for (int k = 0; k < b; ++k) acc -= L[a][k] * L[b][k];
            if (a == b) {
                spd = spd && acc > 0.0;
                L[a][a] = sqrt(acc);
                id[a] = rcp64(L[a][a]);
            } else {
                L[a][b] = acc * id[b];
            }
        }
    }
    if (!spd) return false;
    auto fwd_sub = [&](const double* g, double* y) {  // y = L^-1 g
#pragma unroll
        for (int a = 0; a < N; ++a) {
            double acc = g[a];
#pragma unroll
            for (int k = 0; k < a; ++k) acc -= L[a][k] * y[k];
            y[a] = acc * id[a];
        }
    };
    double Gy[MP][N], qy[N];
#pragma unroll
    for (int r = 0; r < MP; ++r) {
        double g[N];
#pragma unroll
        for (int k = 0; k < N; ++k) g[k] = (double)Q.G[r][k];
        fwd_sub(g, Gy[r]);
    }
    fwd_sub(Q.q, qy);
    double hy[MP];
#pragma unroll
    for (int r = 0; r < MP; ++r) hy[r] = (double)Q.h[r];
    PMat<N, true> pm;
    double one[N];
#pragma unroll
    for (int k = 0; k < N; ++k) one[k] = 1.0;
    pmat_set_diag<N>(pm, one);
    gi_solve<N, MP, true, double>(pm, qy, Gy, hy, max_iter, res);
    double z[N];
#pragma unroll
    for (int a = N - 1; a >= 0; --a) {  // z = L^-T y
        double acc = res.z[a];
#pragma unroll
        for (int k = a + 1; k < N; ++k) acc -= L[k][a] * z[k];
        z[a] = acc * id[a];
    }
#pragma unroll
    for (int k = 0; k < N; ++k) res.z[k] = z[k];
    return true;
}

// Multipliers and active set of a layer-structured QP from its closed-form
// optimum z (diagonal P, q = 0): the rows with G_r z = h_r (to 1e-9
// relative) form A, and lam_A solves the stationarity condition
// P z + G_A' lam_A = 0 on them (G_A P^-1 G_A' lam_A = -G_A z).  Returns false
// for a degenerate point (more than n rows tight, a negative multiplier or a
// stationarity residual), where the caller falls back to Goldfarb-Idnani.
template <int N, int MP, typename T>
__device__ __forceinline__ bool structured_multipliers(const StagedQP<N, MP, T>& Q, int m, QPResult<N, MP>& res) {
    double GA[N][N], ip[N];
#pragma unroll
    for (int k = 0; k < N; ++k) ip[k] = rcp64(Q.P[k][k]);
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
    for (int r = 0; r < MP; ++r) {
        double v = -(double)Q.h[r];
#pragma unroll
        for (int k = 0; k < N; ++k) v = fma((double)Q.G[r][k], res.z[k], v);
        const bool tight = (r < m) && fabs(v) <= 1e-9 * (1.0 + fabs((double)Q.h[r]));
        ok = ok && !(tight && nact >= N);
        const bool a = tight && nact < N;
#pragma unroll
        for (int sl = 0; sl < N; ++sl) {
            const bool here = a && (sl == nact);
#pragma unroll
            for (int k = 0; k < N; ++k) GA[sl][k] = here ? (double)Q.G[r][k] : GA[sl][k];
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
        w[a] = (a < nact) ? -dotd<N>(GA[a], res.z) : 0.0;
    }
    ok = ok && ldl_solve<N>(S, w, lam);
    double scale = 1.0;
#pragma unroll
    for (int sl = 0; sl < N; ++sl) scale = fmax(scale, fabs(lam[sl]));
#pragma unroll
    for (int sl = 0; sl < N; ++sl) ok = ok && (sl >= nact || lam[sl] >= -1e-9 * scale);
#pragma unroll
    for (int k = 0; k < N; ++k) {  // stationarity: P z + G_A' lam = 0
        double acc = Q.P[k][k] * res.z[k];
#pragma unroll
        for (int sl = 0; sl < N; ++sl) acc = fma((sl < nact) ? GA[sl][k] : 0.0, lam[sl], acc);
        ok = ok && fabs(acc) <= 1e-7 * scale * (1.0 + fabs(Q.P[k][k] * res.z[k]));
    }
#pragma unroll
    for (int r = 0; r < MP; ++r) {
        double l = 0.0;
#pragma unroll
        for (int sl = 0; sl < N; ++sl) l = (sl < nact && aidx[sl] == r) ? fmax(lam[sl], 0.0) : l;
        res.lam[r] = l;
    }
    res.active = amask;
    res.nact = nact;
    return ok;
}

// The backward of a layer-structured QP at its closed-form optimum z
// (diagonal P, q = 0) from ONE factorisation: the tight rows A (as
// structured_multipliers), S = G_A P^-1 G_A' (LDL^T), then
//   lam_A = S^-1 (-G_A z)               (stationarity P z + G_A' lam_A = 0)
//   eta   = S^-1 (-G_A P^-1 g),  dz = -P^-1 (g + G_A' eta)   (qp_adjoint)
// -- at a vertex (|A| = n) this is eta = -G_A'^-1 g, dz = 0.  Returns false
// where structured_multipliers would (the caller then runs Goldfarb-Idnani and
// qp_adjoint).
template <int N, int MP, typename T>
__device__ __forceinline__ bool structured_kkt_adjoint(const StagedQP<N, MP, T>& Q, int m, const double* g,
                                                       QPResult<N, MP>& res, double* dz, double* eta, int* aidx) {
    double GA[N][N], ip[N];
#pragma unroll
    for (int k = 0; k < N; ++k) ip[k] = rcp64(Q.P[k][k]);
    int nact = 0;
    uint32_t amask = 0;
    bool ok = true;
    T GAt[N][N];  // the tight rows, gathered in the rows' own type (one select per entry)
#pragma unroll
    for (int sl = 0; sl < N; ++sl) {
        aidx[sl] = -1;
#pragma unroll
        for (int k = 0; k < N; ++k) GAt[sl][k] = T(0);
    }
#pragma unroll
    for (int r = 0; r < MP; ++r) {
        double v = -(double)Q.h[r];
#pragma unroll
        for (int k = 0; k < N; ++k) v = fma((double)Q.G[r][k], res.z[k], v);
        const bool tight = (r < m) && fabs(v) <= 1e-9 * (1.0 + fabs((double)Q.h[r]));
        ok = ok && !(tight && nact >= N);
        const bool a = tight && nact < N;
#pragma unroll
        for (int sl = 0; sl < N && sl <= r; ++sl) {  // row r can only land in slots 0..r
            const bool here = a && (sl == nact);
#pragma unroll
            for (int k = 0; k < N; ++k) GAt[sl][k] = here ? Q.G[r][k] : GAt[sl][k];
            aidx[sl] = here ? r : aidx[sl];
        }
        amask |= a ? (1u << r) : 0u;
        nact += a ? 1 : 0;
    }
#pragma unroll
    for (int sl = 0; sl < N; ++sl)
#pragma unroll
        for (int k = 0; k < N; ++k) GA[sl][k] = (double)GAt[sl][k];
    double S[N][N], w1[N], w2[N], lam[N], Pg[N];
#pragma unroll
    for (int k = 0; k < N; ++k) Pg[k] = ip[k] * g[k];
#pragma unroll
    for (int a = 0; a < N; ++a) {
#pragma unroll
        for (int b = 0; b <= a; ++b) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < N; ++k) acc = fma(GA[a][k] * ip[k], GA[b][k], acc);
            S[a][b] = (a < nact && b < nact) ? acc : (a == b ? 1.0 : 0.0);
            S[b][a] = S[a][b];
        }
        w1[a] = (a < nact) ? -dotd<N>(GA[a], res.z) : 0.0;
        w2[a] = (a < nact) ? -dotd<N>(GA[a], Pg) : 0.0;
    }
    ok = ok && ldl_solve2<N>(S, w1, w2, lam, eta);
    double scale = 1.0;
#pragma unroll
    for (int sl = 0; sl < N; ++sl) scale = fmax(scale, fabs(lam[sl]));
#pragma unroll
    for (int sl = 0; sl < N; ++sl) ok = ok && (sl >= nact || lam[sl] >= -1e-9 * scale);
#pragma unroll
    for (int k = 0; k < N; ++k) {  // stationarity: P z + G_A' lam = 0;  dz = -P^-1 (g + G_A' eta)
        double acc = Q.P[k][k] * res.z[k], t = g[k];
#pragma unroll
        for (int sl = 0; sl < N; ++sl) {
            acc = fma((sl < nact) ? GA[sl][k] : 0.0, lam[sl], acc);
            t = fma((sl < nact) ? GA[sl][k] : 0.0, eta[sl], t);
        }
        ok = ok && fabs(acc) <= 1e-7 * scale * (1.0 + fabs(Q.P[k][k] * res.z[k]));
        dz[k] = -ip[k] * t;
    }
#pragma unroll
    for (int sl = 0; sl < N; ++sl) eta[sl] = (sl < nact) ? eta[sl] : 0.0;
#pragma unroll
    for (int r = 0; r < MP; ++r) {
        double l = 0.0;
#pragma unroll
        for (int sl = 0; sl < N; ++sl) l = (sl < nact && aidx[sl] == r) ? fmax(lam[sl], 0.0) : l;
        res.lam[r] = l;
    }
    res.active = amask;
    res.nact = nact;
    return ok;
}

// Generic QP: rows padded to MP with the never-active row (0 z <= 1); SPD P
// (n <= 3).  T = float: the fp32 rows of the diff layer (z returned as fp32,
// the reference's .float()); T = double: fp64 throughout.  Per wave: the
// layer-structured fast path (exact closed-form solvers) when every lane has
// that structure and no multipliers are asked for; else the diagonal-P or
// full-P Goldfarb-Idnani (or PDIPM) solver.
template <int SOLVER, int N, int MP, typename T>
__global__ void __launch_bounds__(kQPBlock) k_qp_solve(rcbf_params prm, int64_t B, int m, const T* __restrict__ P,
                                                       const T* __restrict__ q, const T* __restrict__ G,
                                                       const T* __restrict__ h, int normalize,
                                                       T* __restrict__ z_out, double* __restrict__ lam_out,
                                                       int32_t* __restrict__ status_out, int32_t* fail_flag,
                                                       double* __restrict__ z64_out) {
    extern __shared__ __align__(16) unsigned char qp_smem[];
    T* sG = reinterpret_cast<T*>(qp_smem);
    T* sh = sG + kQPBlock * odd_stride(m * N);
    T* sP = sh + kQPBlock * odd_stride(m);
    T* sq = sP + kQPBlock * odd_stride(N * N);
    const int64_t i0 = (int64_t)blockIdx.x * kQPBlock;
    const int nb = (int)((B - i0) < kQPBlock ? (B - i0) : kQPBlock);
    stage_in<T, MP * N>(G + i0 * m * N, sG, nb, m * N);
    stage_in<T, MP>(h + i0 * m, sh, nb, m);
    stage_in<T, N * N>(P + i0 * N * N, sP, nb, N * N);
    if (q) stage_in<T, N>(q + i0 * N, sq, nb, N);
    __syncthreads();
    const int lane = threadIdx.x;
    if (lane >= nb) return;
    const int64_t i = i0 + lane;
    StagedQP<N, MP, T> Q;
    staged_read<N, MP, T>(sG, sh, sP, sq, lane, m, q != nullptr, Q);
    T Nrm[MP];
    if (normalize) normalize_rows<N, MP, T>(Q.G, Q.h, Nrm, nullptr);
    QPResult<N, MP> res;
    const bool all_diag = __ballot(!Q.diag) == 0;
    bool solved = false;
    if constexpr (SOLVER != RCBF_SOLVER_PDIPM) {
        if (!lam_out && __ballot(!layer_structured<N, MP, T>(Q, m)) == 0) {
            structured_solve<N, MP, T>(Q, m, res.z, res.status);
            solved = true;
        }
    }
    if (!solved) {
        if (all_diag) {
            PMat<N, true> pm;
            double pd[N];
#pragma unroll
            for (int k = 0; k < N; ++k) pd[k] = Q.P[k][k];
            pmat_set_diag_rt<N>(pm, pd);
            qp_solve<SOLVER, N, MP, true, T>(pm, Q.q, Q.G, Q.h, prm.max_iter, prm.eps, res);
        } else {
            bool done = false;
            if constexpr (SOLVER != RCBF_SOLVER_PDIPM)
                done = gi_solve_chol<N, MP, T>(Q, prm.max_iter > 0 ? prm.max_iter : 4 * (MP + N) + 8, res);
            if (!done) {
                PMat<N, false> pm;
                pmat_set_full<N>(pm, Q.P);
                qp_solve<SOLVER, N, MP, false, T>(pm, Q.q, Q.G, Q.h, prm.max_iter, prm.eps, res);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < N; ++k) z_out[i * N + k] = (T)res.z[k];
    if (z64_out) {
#pragma unroll
        for (int k = 0; k < N; ++k) z64_out[i * N + k] = res.z[k];
    }
    if (lam_out) {
#pragma unroll
        for (int r = 0; r < MP; ++r)
            if (r < m) lam_out[i * m + r] = res.lam[r];
    }
    report(res.status, status_out, i, fail_flag);
}

// dynamic LDS above the default 64 KiB (fp64 staging at m > 12) must be opted into per kernel
inline void allow_lds(const void* kernel, size_t bytes) {
    if (bytes > 65536) (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <typename T>
int qp_solve_launch(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const T* P, const T* q, const T* G,
                    const T* h, int32_t normalize, T* z_out, double* lam_out, int32_t* status_out,
                    int32_t* fail_flag, hipStream_t stream, double* z64_out = nullptr) {
    if (!prm) return RCBF_E_NULL;
    if (prm->solver != RCBF_SOLVER_ACTIVE_SET && prm->solver != RCBF_SOLVER_PDIPM && prm->solver != RCBF_SOLVER_GI)
        return RCBF_E_BAD_MODE;
    if (B < 0 || n < 1 || n > 3 || m < 1 || m > 16) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!P || !G || !h || !z_out) return RCBF_E_NULL;
    dim3 g((unsigned)((B + kQPBlock - 1) / kQPBlock)), b(kQPBlock);
    const size_t lds = (size_t)qp_lds_words(n, m) * sizeof(T);
#define RCBF_QP_L(NN, MP)                                                                                         \
    do {                                                                                                          \
        if (prm->solver == RCBF_SOLVER_PDIPM) {                                                                   \
            allow_lds(reinterpret_cast<const void*>(&k_qp_solve<RCBF_SOLVER_PDIPM, NN, MP, T>), lds);             \
            hipLaunchKernelGGL((k_qp_solve<RCBF_SOLVER_PDIPM, NN, MP, T>), g, b, lds, stream, *prm, B, m, P, q,  \
                               G, h, normalize, z_out, lam_out, status_out, fail_flag, z64_out);                  \
        } else {                                                                                                  \
            allow_lds(reinterpret_cast<const void*>(&k_qp_solve<RCBF_SOLVER_GI, NN, MP, T>), lds);                \
            hipLaunchKernelGGL((k_qp_solve<RCBF_SOLVER_GI, NN, MP, T>), g, b, lds, stream, *prm, B, m, P, q, G,  \
                               h, normalize, z_out, lam_out, status_out, fail_flag, z64_out);                     \
        }                                                                                                         \
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
    // the unicycle layer's rows at the reference's hazard counts 3 and 5 (m = 7, 9) get
    // exact-size instantiations: no padding row in any per-row loop
    if (sizeof(T) == 4 && n == 3 && m == 7)
        RCBF_QP_L(3, 7);
    else if (sizeof(T) == 4 && n == 3 && m == 9)
        RCBF_QP_L(3, 9);
    else if (n == 1)
        RCBF_QP_M(1);
    else if (n == 2)
        RCBF_QP_M(2);
    else
        RCBF_QP_M(3);
#undef RCBF_QP_M
#undef RCBF_QP_L
    return launch_status();
}

}  // namespace rcbf_qp
