// rcbf_device.hpp -- device building blocks of the MI355X batched safe-env step.
//
// One env / one QP per lane.  Everything an env needs lives in VGPRs for the
// whole step: its state, its CBF constraint rows, the QP iterate and the
// active set.  The QP is tiny (n <= 3 variables, m <= 12 rows), so there is
// no MFMA shape here; the kernels are HBM/latency bound and the solvers are
// written branch-light with compile-time loop bounds so every small array
// stays in registers (no scratch).
//
// Numerics mirror the reference's dtypes and operation order:
//   * CBFQPLayer rows: fp32, every elementwise op rounded (torch CPU), no FMA
//     contraction (`#pragma clang fp contract(off)` in those functions)
//   * the QP: fp64 (diff_cbf_qp.py:139 casts to double)
//   * the envs: fp64 (numpy), again without contraction
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rcbf_hip.h"

namespace rcbf {

constexpr double kInf = __builtin_huge_val();


// Study build only (csrc/study/rcbf_stamps.hip defines RCBF_STUDY_QP_STAMPS
// and the buffer): a 16-word record per wave of the unicycle QP -- s_memtime
// at its stage boundaries (slots 0-4) and lane counts (slots 5-8), for
// scripts/stamps.py.  Compiles to nothing in the product.
#ifdef RCBF_STUDY_QP_STAMPS
__device__ __forceinline__ void qp_stamp(int j) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if ((threadIdx.x & 63) == 0 && rcbf_qp_stamp_buf)
        rcbf_qp_stamp_buf[((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + j] = t;
}
__device__ __forceinline__ void qp_count(int j, bool f) {
    const unsigned long long n = __popcll(__ballot(f));
    if ((threadIdx.x & 63) == 0 && rcbf_qp_stamp_buf)
        rcbf_qp_stamp_buf[((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + j] = n;
}
#define RCBF_QP_STAMP(j) ::rcbf::qp_stamp(j)
#define RCBF_QP_COUNT(j, f) ::rcbf::qp_count(j, f)
#else
#define RCBF_QP_STAMP(j) ((void)0)
#define RCBF_QP_COUNT(j, f) ((void)0)
#endif

// fp64 reciprocal: v_rcp_f64 + two Newton steps (error ~1 ulp), no
// div_scale/div_fixup chain.  rcp64(0) = inf.
// 1/d to ~11 ulp (one Newton step on v_rcp_f64, which alone is ~2^-24
// accurate; measured, profiles/r01/ubench_fp64.txt): for the QP solvers'
// candidate points, where a few ulps are far inside every tolerance.  The
// bit-exact fp32 row normalisation keeps rcp64 (two steps, 0 ulp measured).
__device__ __forceinline__ double rcp64_qp(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    return (d == 0.0) ? __builtin_copysign(__builtin_huge_val(), d) : r;
}

__device__ __forceinline__ double rcp64(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    return (d == 0.0) ? __builtin_copysign(__builtin_huge_val(), d) : r;
}

// The same two reciprocals without the d == 0 case (5 VALU fewer each; for
// d = 0 they return NaN instead of inf).  For callers whose divisor is never
// 0, or whose d = 0 result is discarded or multiplies a numerator that is 0
// then too (0 * inf and 0 * NaN are both NaN): bit-identical results.
__device__ __forceinline__ double rcp64_qp_nz(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

__device__ __forceinline__ double rcp64_nz(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

// ---------------------------------------------------------------------------
// small fixed-size linear algebra (compile-time sizes -> registers)
// (solver intermediates use rcp64: they are our own algorithm's quantities,
// and the final results are exact KKT solutions either way)
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ double dotd(const double* a, const double* b) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) s = fma(a[k], b[k], s);
    return s;
}

// Solve S r = w for SPD S (N x N, lower triangle used) by LDL^T without
// pivoting.  Padded (inactive) slots carry an identity block.  Returns false
// on a non-positive pivot.
template <int N>
__device__ __forceinline__ bool ldl_solve(double S[N][N], const double* w, double* r) {
    double L[N][N];
    double D[N], Dinv[N];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double d = S[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k] * D[k];
        ok = ok && (d > 0.0);
        D[j] = d;
        double inv = rcp64(d);
        Dinv[j] = inv;
#pragma unroll
        for (int i = j + 1; i < N; ++i) {
            double v = S[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k] * D[k];
            L[i][j] = v * inv;
        }
    }
    double y[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double v = w[i];
#pragma unroll
        for (int k = 0; k < i; ++k) v -= L[i][k] * y[k];
        y[i] = v;
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        double v = y[i] * Dinv[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k) v -= L[k][i] * r[k];
        r[i] = v;
    }
    return ok;
}

// The same LDL^T factorisation applied to two right-hand sides.
template <int N>
__device__ __forceinline__ bool ldl_solve2(double S[N][N], const double* w1, const double* w2, double* r1,
                                           double* r2) {
    double L[N][N];
    double D[N], Dinv[N];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double d = S[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k] * D[k];
        ok = ok && (d > 0.0);
        D[j] = d;
        double inv = rcp64(d);
        Dinv[j] = inv;
#pragma unroll
        for (int i = j + 1; i < N; ++i) {
            double v = S[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k] * D[k];
            L[i][j] = v * inv;
        }
    }
    double y1[N], y2[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double v1 = w1[i], v2 = w2[i];
#pragma unroll
        for (int k = 0; k < i; ++k) {
            v1 -= L[i][k] * y1[k];
            v2 -= L[i][k] * y2[k];
        }
        y1[i] = v1;
        y2[i] = v2;
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        double v1 = y1[i] * Dinv[i], v2 = y2[i] * Dinv[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k) {
            v1 -= L[k][i] * r1[k];
            v2 -= L[k][i] * r2[k];
        }
        r1[i] = v1;
        r2[i] = v2;
    }
    return ok;
}

// Solve A x = b (N x N general, rows of A = active constraint normals) by
// Gaussian elimination with partial pivoting, fully unrolled.
template <int N>
__device__ __forceinline__ void gauss_solve(double A[N][N], double* b, double* x) {
    double pinv[N];
#pragma unroll
    for (int c = 0; c < N; ++c) {
        // pivot: swap the largest |A[r][c]|, r >= c, into row c (select-based)
#pragma unroll
        for (int r = c + 1; r < N; ++r) {
            bool sw = fabs(A[r][c]) > fabs(A[c][c]);
#pragma unroll
            for (int k = 0; k < N; ++k) {
                double a = A[c][k], bb = A[r][k];
                A[c][k] = sw ? bb : a;
                A[r][k] = sw ? a : bb;
            }
            double a = b[c], bb = b[r];
            b[c] = sw ? bb : a;
            b[r] = sw ? a : bb;
        }
        double inv = rcp64(A[c][c]);
        pinv[c] = inv;
#pragma unroll
        for (int r = c + 1; r < N; ++r) {
            double f = A[r][c] * inv;
#pragma unroll
            for (int k = c; k < N; ++k) A[r][k] -= f * A[c][k];
            b[r] -= f * b[c];
        }
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        double v = b[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k) v -= A[i][k] * x[k];
        x[i] = v * pinv[i];
    }
}

// fp32 a / b, correctly rounded, via one fp64 reciprocal of b: the fp64
// product a * rcp64(b) is within ~2^-52 (relative) of a/b, while a quotient
// of two 24-bit significands is never within 2^-48 of an fp32 rounding
// midpoint, so rounding it to fp32 gives RN32(a/b) -- bit-identical to the
// IEEE division torch performs.  Lets a row share one reciprocal.
__device__ __forceinline__ float div_f32_via_rcp(float a, double rb) { return (float)((double)a * rb); }

// sin(x) for |x| <= 1.3 by its Taylor series to x^21 (truncation < 2e-19,
// ~1 ulp rounding), else the library sin.  The cars lead-car term
// sin(0.2 t) stays below 1.3 for t <= 6.5 s, i.e. within one 300-step episode.
__device__ __forceinline__ double sin_small(double x) {
    if (!(fabs(x) <= 1.3)) return sin(x);
    const double x2 = x * x;
    double p = -1.9572941063391263e-20;  // -1/21!
    p = fma(p, x2, 8.2206352466243297e-18);   // 1/19!
    p = fma(p, x2, -2.8114572543455206e-15);  // -1/17!
    p = fma(p, x2, 7.6471637318198164e-13);   // 1/15!
    p = fma(p, x2, -1.6059043836821613e-10);  // -1/13!
    p = fma(p, x2, 2.5052108385441720e-08);   // 1/11!
    p = fma(p, x2, -2.7557319223985893e-06);  // -1/9!
    p = fma(p, x2, 1.9841269841269841e-04);   // 1/7!
    p = fma(p, x2, -8.3333333333333332e-03);  // -1/5!
    p = fma(p, x2, 1.6666666666666666e-01);   // 1/3!  (sign applied below)
    return fma(-x * x2, p, x);
}

// ---------------------------------------------------------------------------
// Strictly convex QP   min 1/2 z'Pz + q'z   s.t.  G z <= h
// P is given by its inverse (diagonal or full, n <= 3).
// ---------------------------------------------------------------------------
template <int N, bool DIAG>
struct PMat {
    double P[N][N];     // P      (only the diagonal when DIAG)
    double Pinv[N][N];  // P^-1   (only the diagonal when DIAG)
    __device__ __forceinline__ void inv_apply(const double* v, double* o) const {
        if (DIAG) {
#pragma unroll
            for (int i = 0; i < N; ++i) o[i] = Pinv[i][i] * v[i];
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i) o[i] = dotd<N>(Pinv[i], v);
        }
    }
    __device__ __forceinline__ void apply(const double* v, double* o) const {
        if (DIAG) {
#pragma unroll
            for (int i = 0; i < N; ++i) o[i] = P[i][i] * v[i];
        } else {
#pragma unroll
            for (int i = 0; i < N; ++i) o[i] = dotd<N>(P[i], v);
        }
    }
};

template <int N>
__device__ __forceinline__ void pmat_set_diag(PMat<N, true>& pm, const double* d) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        pm.P[i][i] = d[i];
        pm.Pinv[i][i] = 1.0 / d[i];  // compile-time constants in the fused kernels: folded
    }
}

// the same for a run-time diagonal (the generic QP kernels): one reciprocal
// instead of an IEEE division sequence each
template <int N>
__device__ __forceinline__ void pmat_set_diag_rt(PMat<N, true>& pm, const double* d) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        pm.P[i][i] = d[i];
        pm.Pinv[i][i] = rcp64(d[i]);
    }
}

// Full SPD P: invert by Gauss-Jordan on the unit vectors (n <= 3).
template <int N>
__device__ __forceinline__ void pmat_set_full(PMat<N, false>& pm, const double Pin[N][N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        double A[N][N], e[N], col[N];
#pragma unroll
        for (int r = 0; r < N; ++r) {
#pragma unroll
            for (int c = 0; c < N; ++c) A[r][c] = Pin[r][c];
            e[r] = (r == j) ? 1.0 : 0.0;
        }
        gauss_solve<N>(A, e, col);
#pragma unroll
        for (int r = 0; r < N; ++r) pm.Pinv[r][j] = col[r];
    }
#pragma unroll
    for (int r = 0; r < N; ++r)
#pragma unroll
        for (int c = 0; c < N; ++c) pm.P[r][c] = Pin[r][c];
}

template <int N, int M>
struct QPResult {
    double z[N];
    double lam[M];     // multipliers (0 for inactive rows)
    uint32_t active;   // bit r set <=> row r in the final active set
    int nact;
    int status;        // RCBF_QP_*
    int iters;
    bool certified;    // PDIPM: the polished point passed the KKT check
};

// Active rows are tracked in N slots (|A| <= n for a strictly convex QP with
// independent active normals).  Slot s holds a copy of its row.
template <int N>
struct ActiveSet {
    double g[N][N];
    double h[N];
    double lam[N];
    int idx[N];
    int n;
};

// Equality-constrained re-solve on the active set ("polish"): the exact KKT
// point for the final active set, recomputed from scratch so the GI step
// accumulation error does not survive.  Vertex case (|A| = n) solves
// G_A z = h_A directly -- well conditioned after row normalisation even when
// the multipliers are ~1e7 (Cascade unicycle, P = diag(10,1e-4,1e7)).
template <int N, bool DIAG>
__device__ __forceinline__ void polish(const PMat<N, DIAG>& pm, const double* x0, const double* q,
                                       ActiveSet<N>& A, double* z) {
    if (A.n == N) {
        double GA[N][N], hA[N];
#pragma unroll
        for (int s = 0; s < N; ++s) {
#pragma unroll
            for (int k = 0; k < N; ++k) GA[s][k] = A.g[s][k];
            hA[s] = A.h[s];
        }
        gauss_solve<N>(GA, hA, z);
        // lam_A = -G_A^{-T} (P z + q)
        double Pz[N], rhs[N], GT[N][N];
        pm.apply(z, Pz);
#pragma unroll
        for (int k = 0; k < N; ++k) rhs[k] = -(Pz[k] + q[k]);
#pragma unroll
        for (int r = 0; r < N; ++r)
#pragma unroll
            for (int c = 0; c < N; ++c) GT[r][c] = A.g[c][r];
        double lam[N];
        gauss_solve<N>(GT, rhs, lam);
#pragma unroll
        for (int s = 0; s < N; ++s) A.lam[s] = lam[s];
        return;
    }
    // |A| < n: lam = S^-1 (G_A x0 - h_A), z = x0 - P^-1 G_A' lam  (+1 refinement)
    double PG[N][N];  // P^-1 g_s
#pragma unroll
    for (int s = 0; s < N; ++s) pm.inv_apply(A.g[s], PG[s]);
    double S[N][N], w[N], lam[N];
#pragma unroll
    for (int s = 0; s < N; ++s) {
#pragma unroll
        for (int t = 0; t < N; ++t) {
            bool in = (s < A.n) && (t < A.n);
            S[s][t] = in ? dotd<N>(A.g[s], PG[t]) : (s == t ? 1.0 : 0.0);
        }
        w[s] = (s < A.n) ? dotd<N>(A.g[s], x0) - A.h[s] : 0.0;
    }
    double S2[N][N];
#pragma unroll
    for (int s = 0; s < N; ++s)
#pragma unroll
        for (int t = 0; t < N; ++t) S2[s][t] = S[s][t];
    ldl_solve<N>(S2, w, lam);
    double res[N], corr[N];
#pragma unroll
    for (int s = 0; s < N; ++s) res[s] = w[s] - dotd<N>(S[s], lam);
#pragma unroll
    for (int s = 0; s < N; ++s)
#pragma unroll
        for (int t = 0; t < N; ++t) S2[s][t] = S[s][t];
    ldl_solve<N>(S2, res, corr);
#pragma unroll
    for (int s = 0; s < N; ++s) lam[s] = (s < A.n) ? lam[s] + corr[s] : 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        double acc = x0[k];
#pragma unroll
        for (int s = 0; s < N; ++s) acc -= PG[s][k] * lam[s];
        z[k] = acc;
    }
#pragma unroll
    for (int s = 0; s < N; ++s) A.lam[s] = lam[s];
}

// Goldfarb-Idnani dual active-set method (the algorithm of quadprog, which
// the reference's CascadeCBFLayer calls at cbf_qp.py:276), in a re-solve
// form suited to n <= 3: the active-set Schur system S = G_A P^-1 G_A' is
// rebuilt and LDL-solved at each step instead of carrying QR updates.
// Rows are type R (fp32 normalised rows of the diff layer, or fp64).
// Starting from the unconstrained minimum, the most violated row is added;
// a partial step drops the blocking active row; every step keeps dual
// feasibility, and the method terminates at the unique optimum.
template <int N, int M, bool DIAG, typename R>
__device__ __forceinline__ void gi_solve(const PMat<N, DIAG>& pm, const double* q, const R (*G)[N],
                                         const R* h, int max_iter, QPResult<N, M>& out) {
    double x0[N];
    pm.inv_apply(q, x0);
#pragma unroll
    for (int k = 0; k < N; ++k) x0[k] = -x0[k];
    double x[N];
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = x0[k];
    ActiveSet<N> A;
    A.n = 0;
#pragma unroll
    for (int s = 0; s < N; ++s) {
        A.idx[s] = -1;
        A.lam[s] = 0.0;
        A.h[s] = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) A.g[s][k] = 0.0;
    }
    uint32_t amask = 0;
    int status = RCBF_QP_MAX_ITER;
    int it = 0;
    bool finite = true;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        finite = finite && isfinite((double)h[r]);
#pragma unroll
        for (int k = 0; k < N; ++k) finite = finite && isfinite((double)G[r][k]);
    }
    if (!finite) {
        status = RCBF_QP_NONFINITE;
        it = max_iter;
    }
    while (it < max_iter) {
        // (1) most violated inactive row
        int p = -1;
        double vbest = 0.0;
        double gp[N], hp = 0.0;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            double gr[N];
#pragma unroll
            for (int k = 0; k < N; ++k) gr[k] = (double)G[r][k];
            double v = dotd<N>(gr, x) - (double)h[r];
            double tol = 1e-12 * (1.0 + fabs((double)h[r]));
            bool take = !((amask >> r) & 1u) && (v > tol) && (v > vbest);
            vbest = take ? v : vbest;
            p = take ? r : p;
#pragma unroll
            for (int k = 0; k < N; ++k) gp[k] = take ? gr[k] : gp[k];
            hp = take ? (double)h[r] : hp;
        }
        if (p < 0) {
            status = RCBF_QP_OK;
            break;
        }
        double lamp = 0.0;
        // (2) step loop for the violated row p
        bool added = false;
        while (it < max_iter) {
            ++it;
            double Pg[N];
            pm.inv_apply(gp, Pg);
            double PG[N][N];
#pragma unroll
            for (int s = 0; s < N; ++s) pm.inv_apply(A.g[s], PG[s]);
            double S[N][N], w[N], r[N];
#pragma unroll
            for (int s = 0; s < N; ++s) {
#pragma unroll
                for (int t = 0; t < N; ++t) {
                    bool in = (s < A.n) && (t < A.n);
                    S[s][t] = in ? dotd<N>(A.g[s], PG[t]) : (s == t ? 1.0 : 0.0);
                }
                w[s] = (s < A.n) ? dotd<N>(A.g[s], Pg) : 0.0;
            }
            ldl_solve<N>(S, w, r);
            // primal direction z = -P^-1 (g_p - G_A' r)
            double zdir[N];
#pragma unroll
            for (int k = 0; k < N; ++k) {
                double acc = Pg[k];
#pragma unroll
                for (int s = 0; s < N; ++s) acc -= PG[s][k] * ((s < A.n) ? r[s] : 0.0);
                zdir[k] = -acc;
            }
            double gz = dotd<N>(gp, zdir);
            double gPg = dotd<N>(gp, Pg);
            double t2 = kInf;
            if (A.n < N && gz < -1e-13 * gPg) t2 = (dotd<N>(gp, x) - hp) * rcp64(-gz);
            double t1 = kInf;
            int kdrop = -1;
#pragma unroll
            for (int s = 0; s < N; ++s) {
                bool cand = (s < A.n) && (r[s] > 1e-14);
                double tt = cand ? A.lam[s] * rcp64(r[s]) : kInf;
                bool better = cand && (tt < t1);
                t1 = better ? tt : t1;
                kdrop = better ? s : kdrop;
            }
            if (t1 == kInf && t2 == kInf) {
                status = RCBF_QP_INFEASIBLE;
                it = max_iter;
                break;
            }
            double t = fmin(t1, t2);
            if (t2 != kInf) {
#pragma unroll
                for (int k = 0; k < N; ++k) x[k] = fma(t, zdir[k], x[k]);
            }
#pragma unroll
            for (int s = 0; s < N; ++s) A.lam[s] = (s < A.n) ? fmax(A.lam[s] - t * r[s], 0.0) : 0.0;
            lamp += t;
            if (t2 <= t1) {
                // full step: p joins the active set in slot A.n
#pragma unroll
                for (int s = 0; s < N; ++s) {
                    bool here = (s == A.n);
#pragma unroll
                    for (int k = 0; k < N; ++k) A.g[s][k] = here ? gp[k] : A.g[s][k];
                    A.h[s] = here ? hp : A.h[s];
                    A.lam[s] = here ? lamp : A.lam[s];
                    A.idx[s] = here ? p : A.idx[s];
                }
                A.n += 1;
                amask |= (1u << p);
                added = true;
                break;
            }
            // partial step: drop the blocking row kdrop (shift slots down)
            int dropped = A.idx[0];
#pragma unroll
            for (int s = 0; s < N; ++s) dropped = (s == kdrop) ? A.idx[s] : dropped;
            amask &= ~(1u << dropped);
#pragma unroll
            for (int s = 0; s + 1 < N; ++s) {
                bool sh = (s >= kdrop);
#pragma unroll
                for (int k = 0; k < N; ++k) A.g[s][k] = sh ? A.g[s + 1][k] : A.g[s][k];
                A.h[s] = sh ? A.h[s + 1] : A.h[s];
                A.lam[s] = sh ? A.lam[s + 1] : A.lam[s];
                A.idx[s] = sh ? A.idx[s + 1] : A.idx[s];
            }
            A.n -= 1;
            A.idx[N - 1] = -1;
            A.lam[N - 1] = 0.0;
        }
        (void)added;
    }
    if (status == RCBF_QP_OK) {
        polish<N, DIAG>(pm, x0, q, A, x);
    }
    bool okf = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        out.z[k] = x[k];
        okf = okf && isfinite(x[k]);
    }
    if (!okf && status == RCBF_QP_OK) status = RCBF_QP_NONFINITE;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        double l = 0.0;
#pragma unroll
        for (int s = 0; s < N; ++s) l = (s < A.n && A.idx[s] == r) ? A.lam[s] : l;
        out.lam[r] = l;
    }
    out.active = amask;
    out.nact = A.n;
    out.status = status;
    out.iters = it;
}

// Primal-dual interior point (Mehrotra predictor-corrector), the algorithm
// family of qpth (diff_cbf_qp.py:139; OptNet, Amos & Kolter 2017): slack s,
// multipliers lam, Newton steps on the n x n normal equations
//   (P + G' D G) dx = -rx + G' rs - G' D rz,   D = lam / s,
// qpth's initialisation (s, lam shifted to >= 1), its 0.999 fraction to the
// boundary and sigma = (mu_aff / mu)^3, per-QP best-iterate tracking and its
// stop rule (resid < eps, or notImprovedLim steps without improvement).
// Followed by the same exact active-set polish as the GI path (rows with
// lam > s), so the returned z is the KKT point of the identified set.
template <int N, int M, bool DIAG, typename R>
__device__ __forceinline__ void pdipm_solve(const PMat<N, DIAG>& pm, const double* q, const R (*G)[N],
                                            const R* h, int max_iter, double eps, QPResult<N, M>& out) {
    double Gd[M][N], hd[M];
    bool finite = true;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        hd[r] = (double)h[r];
        finite = finite && isfinite(hd[r]);
#pragma unroll
        for (int k = 0; k < N; ++k) {
            Gd[r][k] = (double)G[r][k];
            finite = finite && isfinite(Gd[r][k]);
        }
    }
    double x[N], s[M], lam[M];
    // initial point: solve the KKT with D = I (qpth's d = ones), rx = q, rz = -h
    {
        double H[N][N];
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
            for (int j = 0; j < N; ++j) {
                double acc = DIAG ? (i == j ? pm.P[i][i] : 0.0) : pm.P[i][j];
#pragma unroll
                for (int r = 0; r < M; ++r) acc += Gd[r][i] * Gd[r][j];
                H[i][j] = acc;
            }
        // (P + G'G) x = -q + G'h   (rs = 0, rz = -h)
        double rhs[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double acc = -q[i];
#pragma unroll
            for (int r = 0; r < M; ++r) acc += Gd[r][i] * hd[r];
            rhs[i] = acc;
        }
        ldl_solve<N>(H, rhs, x);
        double smin = kInf, lmin = kInf;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            double gx = dotd<N>(Gd[r], x);
            // ds = -rz - G dx with rz = -h  ->  s = h - G x ; lam = D(G x - h) = -s
            s[r] = hd[r] - gx;
            lam[r] = gx - hd[r];
            smin = fmin(smin, s[r]);
            lmin = fmin(lmin, lam[r]);
        }
#pragma unroll
        for (int r = 0; r < M; ++r) {
            if (smin < 0.0) s[r] -= smin - 1.0;
            if (lmin < 0.0) lam[r] -= lmin - 1.0;
        }
    }
    double best_res = kInf, bx[N], bs[M], bl[M];
#pragma unroll
    for (int k = 0; k < N; ++k) bx[k] = x[k];
#pragma unroll
    for (int r = 0; r < M; ++r) {
        bs[r] = s[r];
        bl[r] = lam[r];
    }
    int not_improved = 0;
    int it = 0;
    int status = finite ? RCBF_QP_MAX_ITER : RCBF_QP_NONFINITE;
    const int not_improved_lim = 10;  // diff_cbf_qp.py:107
    for (; finite && it < max_iter; ++it) {
        // residuals
        double rx[N], rz[M], Px[N];
        pm.apply(x, Px);
#pragma unroll
        for (int k = 0; k < N; ++k) {
            double acc = Px[k] + q[k];
#pragma unroll
            for (int r = 0; r < M; ++r) acc += Gd[r][k] * lam[r];
            rx[k] = acc;
        }
        double sz = 0.0, zr = 0.0;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            rz[r] = dotd<N>(Gd[r], x) + s[r] - hd[r];
            sz += s[r] * lam[r];
            zr += rz[r] * rz[r];
        }
        double mu = fabs(sz / M);
        double res = sqrt(zr) + sqrt(dotd<N>(rx, rx)) + M * mu;
        if (res < best_res) {
            best_res = res;
            not_improved = 0;
#pragma unroll
            for (int k = 0; k < N; ++k) bx[k] = x[k];
#pragma unroll
            for (int r = 0; r < M; ++r) {
                bs[r] = s[r];
                bl[r] = lam[r];
            }
        } else {
            ++not_improved;
        }
        if (best_res < eps) {
            status = RCBF_QP_OK;
            break;
        }
        if (not_improved >= not_improved_lim) {
            status = RCBF_QP_OK;  // qpth returns its best iterate here too
            break;
        }
        // normal-equation matrix H = P + G' D G
        double d[M], H[N][N];
#pragma unroll
        for (int r = 0; r < M; ++r) d[r] = lam[r] * rcp64(s[r]);
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
            for (int j = 0; j <= i; ++j) {
                double acc = DIAG ? (i == j ? pm.P[i][i] : 0.0) : pm.P[i][j];
#pragma unroll
                for (int r = 0; r < M; ++r) acc += Gd[r][i] * d[r] * Gd[r][j];
                H[i][j] = acc;
                H[j][i] = acc;
            }
        // affine direction: rs = lam
        double dx[N], ds[M], dl[M], rhs[N];
        auto kkt = [&](const double* rs_, double* dx_, double* ds_, double* dl_) {
#pragma unroll
            for (int k = 0; k < N; ++k) {
                double acc = -rx[k];
#pragma unroll
                for (int r = 0; r < M; ++r) acc += Gd[r][k] * (rs_[r] - d[r] * rz[r]);
                rhs[k] = acc;
            }
            double Hc[N][N];
#pragma unroll
            for (int i = 0; i < N; ++i)
#pragma unroll
                for (int j = 0; j < N; ++j) Hc[i][j] = H[i][j];
            ldl_solve<N>(Hc, rhs, dx_);
#pragma unroll
            for (int r = 0; r < M; ++r) {
                ds_[r] = -rz[r] - dotd<N>(Gd[r], dx_);
                dl_[r] = -rs_[r] - d[r] * ds_[r];
            }
        };
        double rs[M];
#pragma unroll
        for (int r = 0; r < M; ++r) rs[r] = lam[r];
        kkt(rs, dx, ds, dl);
        // step to the boundary
        double a_aff = 1.0;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            if (dl[r] < 0.0) a_aff = fmin(a_aff, -lam[r] * rcp64(dl[r]));
            if (ds[r] < 0.0) a_aff = fmin(a_aff, -s[r] * rcp64(ds[r]));
        }
        double t3 = 0.0;
#pragma unroll
        for (int r = 0; r < M; ++r) t3 += (s[r] + a_aff * ds[r]) * (lam[r] + a_aff * dl[r]);
        double sig = t3 * rcp64(sz);
        sig = sig * sig * sig;
        // corrector: rs = (-mu sig + ds_aff dl_aff) / s, rx = rz = 0, added
        double dxc[N], dsc[M], dlc[M];
        {
            double rx0[N], rz0[M];
#pragma unroll
            for (int k = 0; k < N; ++k) {
                rx0[k] = rx[k];
                rx[k] = 0.0;
            }
#pragma unroll
            for (int r = 0; r < M; ++r) {
                rz0[r] = rz[r];
                rz[r] = 0.0;
                rs[r] = (-mu * sig + ds[r] * dl[r]) * rcp64(s[r]);
            }
            kkt(rs, dxc, dsc, dlc);
#pragma unroll
            for (int k = 0; k < N; ++k) rx[k] = rx0[k];
#pragma unroll
            for (int r = 0; r < M; ++r) rz[r] = rz0[r];
        }
        double alpha = 1.0;
#pragma unroll
        for (int k = 0; k < N; ++k) dx[k] += dxc[k];
#pragma unroll
        for (int r = 0; r < M; ++r) {
            ds[r] += dsc[r];
            dl[r] += dlc[r];
        }
        double amax = kInf;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            if (dl[r] < 0.0) amax = fmin(amax, -lam[r] * rcp64(dl[r]));
            if (ds[r] < 0.0) amax = fmin(amax, -s[r] * rcp64(ds[r]));
        }
        // qpth's get_step: no blocking direction -> step 1 (then x0.999)
        if (amax == kInf) amax = 1.0;
        alpha = fmin(1.0, 0.999 * amax);
#pragma unroll
        for (int k = 0; k < N; ++k) x[k] += alpha * dx[k];
#pragma unroll
        for (int r = 0; r < M; ++r) {
            s[r] += alpha * ds[r];
            lam[r] += alpha * dl[r];
        }
    }
    // active-set polish on {r : lam_r > s_r} (at most N rows, largest lam first)
    ActiveSet<N> A;
    A.n = 0;
    uint32_t amask = 0;
#pragma unroll
    for (int sl = 0; sl < N; ++sl) {
        A.idx[sl] = -1;
        A.lam[sl] = 0.0;
        A.h[sl] = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) A.g[sl][k] = 0.0;
    }
#pragma unroll
    for (int sl = 0; sl < N; ++sl) {
        int pick = -1;
        double lb = 0.0;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            bool c = !((amask >> r) & 1u) && (bl[r] > bs[r]) && (bl[r] > lb);
            lb = c ? bl[r] : lb;
            pick = c ? r : pick;
        }
        if (pick >= 0) {
#pragma unroll
            for (int r = 0; r < M; ++r) {
                if (r == pick) {
#pragma unroll
                    for (int k = 0; k < N; ++k) A.g[sl][k] = Gd[r][k];
                    A.h[sl] = hd[r];
                }
            }
            A.idx[sl] = pick;
            A.n = sl + 1;
            amask |= 1u << pick;
        }
    }
    double z[N];
#pragma unroll
    for (int k = 0; k < N; ++k) z[k] = bx[k];
    out.certified = false;
    if (finite) {
        double x0[N];
        pm.inv_apply(q, x0);
#pragma unroll
        for (int k = 0; k < N; ++k) x0[k] = -x0[k];
        double zp[N];
        polish<N, DIAG>(pm, x0, q, A, zp);
        // accept the polish only if it is primal and dual feasible
        bool ok = true;
#pragma unroll
        for (int r = 0; r < M; ++r) ok = ok && (dotd<N>(Gd[r], zp) - hd[r] <= 1e-9 * (1.0 + fabs(hd[r])));
#pragma unroll
        for (int sl = 0; sl < N; ++sl) ok = ok && (sl >= A.n || A.lam[sl] >= -1e-9);
#pragma unroll
        for (int k = 0; k < N; ++k) z[k] = ok ? zp[k] : z[k];
        out.certified = ok;
        if (ok) status = RCBF_QP_OK;  // a certified KKT point is the optimum, however many iterations it took
    }
    bool okf = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        out.z[k] = z[k];
        okf = okf && isfinite(z[k]);
    }
    if (!okf) status = RCBF_QP_NONFINITE;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        double l = 0.0;
#pragma unroll
        for (int sl = 0; sl < N; ++sl) l = (sl < A.n && A.idx[sl] == r) ? A.lam[sl] : l;
        out.lam[r] = l;
    }
    out.active = amask;
    out.nact = A.n;
    out.status = status;
    out.iters = it;
}

// Exact solver for n = 2 variables (the cars QP, z = [u, eps]) with diagonal P
// and q = 0: enumerate the KKT candidates of every row subset of size <= 2
// (the unconstrained minimum, the minimiser on each row's hyperplane, each
// pair's vertex) and keep the primal-feasible one with the smallest
// objective.  The optimum is one of the candidates (it minimises the
// objective on the affine hull of its active set) and is feasible; every
// other feasible candidate has an objective at least as large, so no dual
// test is needed.  All candidates are independent: ~1 + M + M(M-1)/2 short
// fp64 expressions with no loop-carried dependency, which suits a single
// wave per SIMD far better than an iterative active-set loop.
template <int M, typename R>
__device__ __forceinline__ void enum2_solve(const PMat<2, true>& pm, const R (*G)[2], const R* h,
                                            QPResult<2, M>& out) {
    const double pi0 = pm.Pinv[0][0], pi1 = pm.Pinv[1][1];
    const double p0 = pm.P[0][0], p1 = pm.P[1][1];
    double g0[M], g1[M], hh[M];
    bool finite = true;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        g0[r] = (double)G[r][0];
        g1[r] = (double)G[r][1];
        hh[r] = (double)h[r];
        finite = finite && isfinite(g0[r]) && isfinite(g1[r]) && isfinite(hh[r]);
    }
    double best = kInf, bz0 = 0.0, bz1 = 0.0;
    uint32_t bact = 0;
    auto consider = [&](double z0, double z1, uint32_t act, bool valid) {
        bool feas = valid;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            double v = fma(g0[r], z0, fma(g1[r], z1, -hh[r]));
            feas = feas && (v <= 1e-9 * (1.0 + fabs(hh[r])));
        }
        double obj = fma(p0 * z0, z0, p1 * z1 * z1);
        bool take = feas && (obj < best);
        best = take ? obj : best;
        bz0 = take ? z0 : bz0;
        bz1 = take ? z1 : bz1;
        bact = take ? act : bact;
    };
    consider(0.0, 0.0, 0u, true);
#pragma unroll
    for (int r = 0; r < M; ++r) {
        // z = P^-1 g h / (g P^-1 g')
        double nrm = fma(g0[r] * pi0, g0[r], g1[r] * pi1 * g1[r]);
        bool ok = nrm > 1e-300;
        double f = ok ? hh[r] * rcp64(nrm) : 0.0;
        consider(pi0 * g0[r] * f, pi1 * g1[r] * f, 1u << r, ok);
    }
#pragma unroll
    for (int r = 0; r < M; ++r) {
#pragma unroll
        for (int s = r + 1; s < M; ++s) {
            double det = g0[r] * g1[s] - g1[r] * g0[s];
            bool ok = fabs(det) > 1e-12;
            double inv = ok ? rcp64(det) : 0.0;
            double z0 = (hh[r] * g1[s] - hh[s] * g1[r]) * inv;
            double z1 = (g0[r] * hh[s] - g0[s] * hh[r]) * inv;
            consider(z0, z1, (1u << r) | (1u << s), ok);
        }
    }
    out.z[0] = bz0;
    out.z[1] = bz1;
    // multipliers of the chosen set:  P z + G_A' lam = 0
    double Pz0 = p0 * bz0, Pz1 = p1 * bz1;
    int ra = -1, rb = -1;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        bool a = (bact >> r) & 1u;
        rb = (a && ra >= 0 && rb < 0) ? r : rb;
        ra = (a && ra < 0) ? r : ra;
    }
    double ga0 = 0, ga1 = 0, gb0 = 0, gb1 = 0;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        ga0 = (r == ra) ? g0[r] : ga0;
        ga1 = (r == ra) ? g1[r] : ga1;
        gb0 = (r == rb) ? g0[r] : gb0;
        gb1 = (r == rb) ? g1[r] : gb1;
    }
    double la = 0.0, lb = 0.0;
    if (rb >= 0) {  // [ga gb] [la lb]' = -Pz  (2x2, Cramer)
        double det = ga0 * gb1 - gb0 * ga1;
        double idet = rcp64(det);
        la = (-Pz0 * gb1 + Pz1 * gb0) * idet;
        lb = (-ga0 * Pz1 + ga1 * Pz0) * idet;
    } else if (ra >= 0) {
        double nn = ga0 * ga0 + ga1 * ga1;
        la = -(Pz0 * ga0 + Pz1 * ga1) * rcp64(nn);
    }
#pragma unroll
    for (int r = 0; r < M; ++r) out.lam[r] = (r == ra) ? la : ((r == rb) ? lb : 0.0);
    out.active = bact;
    out.nact = (ra >= 0) + (rb >= 0);
    out.iters = 1;
    bool okz = isfinite(bz0) && isfinite(bz1) && best < kInf;
    out.status = !finite ? RCBF_QP_NONFINITE : (okz ? RCBF_QP_OK : RCBF_QP_INFEASIBLE);
}

// Fast exact solver for n = 2: the candidate selection of enum2_solve runs in
// fp32 (twice the fp64 rate, cheap approximate reciprocals), then the chosen
// active set is re-solved in fp64 and its KKT conditions are verified in fp64
// (primal feasibility of every row, non-negative multipliers).  A verified KKT
// point IS the unique optimum, so the result equals enum2_solve's; when the
// certificate fails (fp32 picked a near-tie wrongly) the lane falls back to
// the fp64 enumeration.
template <int M, typename R>
__device__ __forceinline__ void enum2_solve_fast(const PMat<2, true>& pm, const R (*G)[2], const R* h,
                                                 QPResult<2, M>& out) {
    const float pi0 = (float)pm.Pinv[0][0], pi1 = (float)pm.Pinv[1][1];
    const float p0 = (float)pm.P[0][0], p1 = (float)pm.P[1][1];
    float g0[M], g1[M], hh[M];
#pragma unroll
    for (int r = 0; r < M; ++r) {
        g0[r] = (float)G[r][0];
        g1[r] = (float)G[r][1];
        hh[r] = (float)h[r];
    }
    float best = __builtin_huge_valf();
    uint32_t bact = 0;
    auto consider = [&](float z0, float z1, uint32_t act, bool valid) {
        bool feas = valid;
#pragma unroll
        for (int r = 0; r < M; ++r) {
            float v = fmaf(g0[r], z0, fmaf(g1[r], z1, -hh[r]));
            feas = feas && (v <= 1e-5f * (1.0f + fabsf(hh[r])));
        }
        float obj = fmaf(p0 * z0, z0, p1 * z1 * z1);
        bool take = feas && (obj < best);
        best = take ? obj : best;
        bact = take ? act : bact;
    };
    consider(0.0f, 0.0f, 0u, true);
#pragma unroll
    for (int r = 0; r < M; ++r) {
        float nrm = fmaf(g0[r] * pi0, g0[r], g1[r] * pi1 * g1[r]);
        bool ok = nrm > 1e-30f;
        float f = hh[r] * __builtin_amdgcn_rcpf(ok ? nrm : 1.0f);
        consider(pi0 * g0[r] * f, pi1 * g1[r] * f, 1u << r, ok);
    }
#pragma unroll
    for (int r = 0; r < M; ++r) {
#pragma unroll
        for (int s = r + 1; s < M; ++s) {
            float det = fmaf(g0[r], g1[s], -g1[r] * g0[s]);
            bool ok = fabsf(det) > 1e-7f;
            float inv = __builtin_amdgcn_rcpf(ok ? det : 1.0f);
            float z0 = fmaf(hh[r], g1[s], -hh[s] * g1[r]) * inv;
            float z1 = fmaf(g0[r], hh[s], -g0[s] * hh[r]) * inv;
            consider(z0, z1, (1u << r) | (1u << s), ok);
        }
    }
    // fp64 re-solve of the chosen set and its KKT certificate
    int ra = -1, rb = -1;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        bool a = (bact >> r) & 1u;
        rb = (a && ra >= 0 && rb < 0) ? r : rb;
        ra = (a && ra < 0) ? r : ra;
    }
    double ga0 = 0, ga1 = 0, gb0 = 0, gb1 = 0, ha = 0, hb = 0;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        ga0 = (r == ra) ? (double)G[r][0] : ga0;
        ga1 = (r == ra) ? (double)G[r][1] : ga1;
        ha = (r == ra) ? (double)h[r] : ha;
        gb0 = (r == rb) ? (double)G[r][0] : gb0;
        gb1 = (r == rb) ? (double)G[r][1] : gb1;
        hb = (r == rb) ? (double)h[r] : hb;
    }
    const double dpi0 = pm.Pinv[0][0], dpi1 = pm.Pinv[1][1], dp0 = pm.P[0][0], dp1 = pm.P[1][1];
    double z0 = 0.0, z1 = 0.0, la = 0.0, lb = 0.0;
    if (rb >= 0) {
        double det = ga0 * gb1 - ga1 * gb0;
        double inv = 1.0 / det;
        z0 = (ha * gb1 - hb * ga1) * inv;
        z1 = (ga0 * hb - gb0 * ha) * inv;
        double Pz0 = dp0 * z0, Pz1 = dp1 * z1;
        la = (-Pz0 * gb1 + Pz1 * gb0) * inv;
        lb = (-ga0 * Pz1 + ga1 * Pz0) * inv;
    } else if (ra >= 0) {
        double nrm = fma(ga0 * dpi0, ga0, ga1 * dpi1 * ga1);
        double f = ha / nrm;
        z0 = dpi0 * ga0 * f;
        z1 = dpi1 * ga1 * f;
        la = -f;
    }
    bool cert = isfinite(z0) && isfinite(z1) && (la >= -1e-12) && (lb >= -1e-12);
#pragma unroll
    for (int r = 0; r < M; ++r) {
        double v = fma((double)G[r][0], z0, fma((double)G[r][1], z1, -(double)h[r]));
        cert = cert && (v <= 1e-9 * (1.0 + fabs((double)h[r])));
    }
    if (!cert) {  // rare: near-tie mis-selected in fp32 (or non-finite input)
        enum2_solve<M, R>(pm, G, h, out);
        return;
    }
    out.z[0] = z0;
    out.z[1] = z1;
#pragma unroll
    for (int r = 0; r < M; ++r) out.lam[r] = (r == ra) ? la : ((r == rb) ? lb : 0.0);
    out.active = bact;
    out.nact = (ra >= 0) + (rb >= 0);
    out.iters = 0;
    out.status = RCBF_QP_OK;
}

// Exact solver for the CARS QP structure (both formulations):
//   rows 0,1:  g_r0 u + g_r1 eps <= h_r  with g_r1 < 0 (the -200 slack column)
//   row 2:     g_20 u <= h_2  (g_20 > 0)     row 3:  g_30 u <= h_3  (g_30 < 0)
//   objective  1/2 (p0 u^2 + p1 eps^2)
// For a fixed u the best slack is eps*(u) = max(0, e0(u), e1(u)) with the
// affine e_r(u) = (h_r - g_r0 u) / g_r1, so the QP is the 1-D convex problem
// min_{L <= u <= U} phi(u) = p0 u^2 + p1 eps*(u)^2, U = h2/g20, L = h3/g30.
// phi is convex and piecewise quadratic; its unconstrained minimiser is 0
// (eps* = 0 piece), a stationary point of one of the two e_r pieces, or the
// kink e0 = e1 (phi is differentiable where an e_r crosses 0), and the
// constrained minimiser is that point clamped to [L, U].  Evaluating phi
// exactly at the four clamped candidates and keeping the smallest is
// therefore exact -- no feasibility or dual tests, no active-set loop, and
// any extra candidate is harmless (all lie in [L, U]).  ~60 fp64 ops vs
// ~400 for the generic enumeration.  Multipliers are not produced (the
// forward does not need them; the backward uses enum2_solve).
template <typename R>
__device__ __forceinline__ void cars_qp_1d(const PMat<2, true>& pm, const R (*G)[2], const R* h, double* z,
                                           int& status) {
    const double p0 = pm.P[0][0], p1 = pm.P[1][1];
    const double g00 = (double)G[0][0], g01 = (double)G[0][1], h0 = (double)h[0];
    const double g10 = (double)G[1][0], g11 = (double)G[1][1], h1 = (double)h[1];
    const double U = (double)h[2] * rcp64_qp_nz((double)G[2][0]);
    const double L = (double)h[3] * rcp64_qp_nz((double)G[3][0]);
    const double i0 = rcp64_qp_nz(g01), i1 = rcp64_qp_nz(g11);
    const double a0 = -g00 * i0, b0 = h0 * i0;  // e0(u) = a0 u + b0
    const double a1 = -g10 * i1, b1 = h1 * i1;  // e1(u) = a1 u + b1
    const double c1 = -(p1 * a0 * b0) * rcp64_qp_nz(fma(p1 * a0, a0, p0));
    const double c2 = -(p1 * a1 * b1) * rcp64_qp_nz(fma(p1 * a1, a1, p0));
    const double den = a0 - a1;
    const double c3 = (den != 0.0) ? (b1 - b0) * rcp64_qp_nz(den) : 0.0;
    auto clampu = [&](double u) { return fmin(fmax(u, L), U); };
    auto phi = [&](double u) {
        double e = fmax(0.0, fmax(fma(a0, u, b0), fma(a1, u, b1)));
        return fma(p0 * u, u, p1 * e * e);
    };
    double ub = clampu(0.0), fb = phi(ub);
    double u1 = clampu(c1), f1 = phi(u1);
    double u2 = clampu(c2), f2 = phi(u2);
    double u3 = clampu(c3), f3 = phi(u3);
    ub = (f1 < fb) ? u1 : ub;
    fb = fmin(f1, fb);
    ub = (f2 < fb) ? u2 : ub;
    fb = fmin(f2, fb);
    ub = (f3 < fb) ? u3 : ub;
    z[0] = ub;
    z[1] = fmax(0.0, fmax(fma(a0, ub, b0), fma(a1, ub, b1)));
    // fmin/fmax drop NaNs, so non-finite data must be caught on the inputs:
    // the reference's solver returns NaN there and the layer raises (diff_cbf_qp.py:141-143)
    const bool fin = isfinite(g00 + g01 + h0 + g10 + g11 + h1 + U + L + a0 + a1 + b0 + b1);
    const bool ok = fin && isfinite(z[0]) && isfinite(z[1]) && (L <= U);
    status = ok ? RCBF_QP_OK : (fin ? RCBF_QP_INFEASIBLE : RCBF_QP_NONFINITE);
    if (!fin) z[0] = z[1] = __builtin_nan("");
}

// The same exact solver on the cars layer's RAW rows (the fused safe step):
// the reference row-normalises before qpth (diff_cbf_qp.py:103-106), a
// positive scaling of each row that leaves the feasible set, hence the
// exact optimum, unchanged -- so the fused step skips it and solves the rows
// as built.  Rows 0, 1: G_r0 u + G_r1 eps <= h_r with G_r1 = -200 exactly
// (cars_rows_diff); rows 2, 3: u <= h_2, -u <= h_3.  With eps' = 200 eps the
// CBF rows read eps' >= e_r(u) = G_r0 u - h_r and the slack weight is
// p1 / 40000, so e_r's coefficients are the fp32 row entries themselves (no
// division) and the actuator bounds are h_2 and -h_3.  Against the
// normalised problem the optimum moves only by the fp32 rounding of the
// normalised entries (~1e-7 relative), far inside the north star's 1e-4.
template <typename R>
__device__ __forceinline__ void cars_qp_1d_raw(const PMat<2, true>& pm, const R (*G)[2], const R* h, double* z,
                                               int& status) {
    const double p0 = pm.P[0][0], p1 = pm.P[1][1] * (1.0 / 40000.0);
    const double a0 = (double)G[0][0], b0 = -(double)h[0];
    const double a1 = (double)G[1][0], b1 = -(double)h[1];
    const double U = (double)h[2], L = -(double)h[3];
    const double c1 = -(p1 * a0 * b0) * rcp64_qp_nz(fma(p1 * a0, a0, p0));
    const double c2 = -(p1 * a1 * b1) * rcp64_qp_nz(fma(p1 * a1, a1, p0));
    const double den = a0 - a1;
    const double c3 = (den != 0.0) ? (b1 - b0) * rcp64_qp_nz(den) : 0.0;
    auto clampu = [&](double u) { return fmin(fmax(u, L), U); };
    auto phi = [&](double u) {
        double e = fmax(0.0, fmax(fma(a0, u, b0), fma(a1, u, b1)));
        return fma(p0 * u, u, p1 * e * e);
    };
    double ub = clampu(0.0), fb = phi(ub);
    double u1 = clampu(c1), f1 = phi(u1);
    double u2 = clampu(c2), f2 = phi(u2);
    double u3 = clampu(c3), f3 = phi(u3);
    ub = (f1 < fb) ? u1 : ub;
    fb = fmin(f1, fb);
    ub = (f2 < fb) ? u2 : ub;
    fb = fmin(f2, fb);
    ub = (f3 < fb) ? u3 : ub;
    z[0] = ub;
    z[1] = fmax(0.0, fmax(fma(a0, ub, b0), fma(a1, ub, b1))) * (1.0 / 200.0);
    // non-finite rows are caught on the inputs (fmin/fmax drop NaNs); the
    // reference's solver returns NaN there and the layer raises (:141-143)
    const bool fin = isfinite(a0 + b0 + a1 + b1 + U + L + (double)G[0][1] + (double)G[1][1]);
    const bool ok = fin && isfinite(z[0]) && (L <= U);
    status = ok ? RCBF_QP_OK : (fin ? RCBF_QP_INFEASIBLE : RCBF_QP_NONFINITE);
    if (!fin) z[0] = z[1] = __builtin_nan("");
}

// Exact solver for the UNICYCLE QP structure (both formulations), z = (u0, u1, eps):
//   rows j < K:  g_j0 u0 + g_j1 u1 + g_j2 eps <= h_j  with g_j2 < 0 (slack column)
//   rows K..K+3: u0 <= U0, -u0 <= .., u1 <= U1, -u1 <= ..  (the actuator box)
//   objective    1/2 (p0 u0^2 + p1 u1^2 + p2 eps^2)
// As for cars, eps*(u) = max(0, max_j e_j(u)) with affine e_j(u) = a_j.u + b_j,
// leaving the 2-D convex piecewise quadratic
//   phi(u) = p0 u0^2 + p1 u1^2 + p2 eps*(u)^2   over the box.
//
// Pruning (exact): a hazard row whose e_j(u) <= 0 over the WHOLE box never
// changes eps*(u) on the box -- phi on the box, hence the constrained optimum,
// is the same with or without it.  Each lane keeps only its live rows
// (max over the box of a_j.u + b_j > 0, i.e. the hazard can bind), compacted
// into slots; the wave then solves with KK = the largest live count of its
// lanes (a wave-uniform branch), so a lane far from every hazard costs one
// clamp and a typical wave (<= 2 hazards within reach of any of its envs)
// enumerates 2 pieces + 1 kink instead of K + K(K-1)/2 + C(K,3) candidates.
// Unused slots of a lane repeat its first slot (a duplicated piece only adds
// NaN kink / triple candidates, which never win, and duplicate points).
//
// uni_pieces_solve<KK> on the slots:
// Stage 1, box-free optimum: it is u = 0, the stationary point of one piece
// (Sherman-Morrison on diag(p0,p1) + p2 a a'), the minimiser on one kink line
// e_i = e_j, or a triple point e_i = e_j = e_l (phi is differentiable where an
// e_j crosses 0); the argmin of phi over these candidates is exact.
// Certificates let most waves stop after u = 0 and the pieces: phi is convex
// and phi = max_j f_j with f_j = p0 u0^2 + p1 u1^2 + p2 max(0, e_j)^2, so
//   * u = 0 is optimal when every b_j <= 0 (phi(0) = 0 <= phi);
//   * piece j's stationary point u_j is optimal when e_j(u_j) > 0 and piece j
//     attains the max there (ties included): then f_j is active at u_j and
//     grad f_j(u_j) = 0 lies in the subdifferential of phi.
// The kink and triple candidates run only in waves with an uncertified lane
// (a wave-uniform ballot) and only update such lanes.
// Stage 2: if that point u_f leaves the box, the constrained optimum lies on
// a FACING edge -- one whose constraint u_f violates (otherwise a small step
// from it toward u_f stays feasible and strictly lowers phi).  So the u0-edge
// (u0 = clamp(u_f0)) is needed only where u_f0 leaves [L0, U0], the u1-edge
// only where u_f1 leaves [L1, U1]; each is a 1-D problem solved exactly like
// cars_qp_1d (clamped stationary points and kinks, with stage 1's
// certificates), run only in waves with a lane that needs it.  (Stage 2 stays exact for the pruned phi: it equals the full
// phi on the box, and the facing-edge argument holds for any convex function.)
template <int KK>
__device__ __forceinline__ void uni_pieces_solve(double p0, double p1, double p2, double ip0, double ip1,
                                                 const double* a0, const double* a1, const double* b, double L0,
                                                 double U0, double L1, double U1, double& bu0, double& bu1,
                                                 double& bf) {
    auto eps_of = [&](double u0, double u1) {
        double e = 0.0;
#pragma unroll
        for (int j = 0; j < KK; ++j) e = fmax(e, fma(a0[j], u0, fma(a1[j], u1, b[j])));
        return e;
    };
    auto phi_e = [&](double u0, double u1, double e) { return fma(p0 * u0, u0, fma(p1 * u1, u1, p2 * e * e)); };
    bool open = true;  // no certificate yet
    auto take = [&](double u0, double u1) {
        double f = phi_e(u0, u1, eps_of(u0, u1));
        bool t = open && f < bf;  // NaN candidates never win
        bu0 = t ? u0 : bu0;
        bu1 = t ? u1 : bu1;
        bf = t ? f : bf;
    };
    // stage 2's 1-D problem on an edge: the fixed coordinate at v, the free one
    // y in [lo, hi]; e_j = al_j y + be_j and phi(y) = pf y^2 + (p_fixed v^2 +
    // p2 eps(y)^2), convex, whose minimiser is the clamp of the unconstrained
    // one, certified like stage 1 (origin: every be_j <= 0; piece j: e_j(y_j) > 0
    // is the max) -> (ey, ef); nd gates its kink candidates by ballot
    auto edge_solve = [&](bool fix0, double v, double lo, double hi, bool nd, double& ey, double& ef) {
        double al[KK], be[KK];
        bool eneg = true;
#pragma unroll
        for (int j = 0; j < KK; ++j) {
            al[j] = fix0 ? a1[j] : a0[j];
            be[j] = fix0 ? fma(a0[j], v, b[j]) : fma(a1[j], v, b[j]);
            eneg = eneg && (be[j] <= 0.0);
        }
        const double pf = fix0 ? p1 : p0;
        const double cfix = (fix0 ? p0 : p1) * v * v;
        auto emax = [&](double y) {
            double e = 0.0;
#pragma unroll
            for (int j = 0; j < KK; ++j) e = fmax(e, fma(al[j], y, be[j]));
            return e;
        };
        auto fval = [&](double y) {
            const double e = emax(y);
            return fma(pf * y, y, fma(p2 * e, e, cfix));
        };
        ey = fmin(fmax(0.0, lo), hi);
        ef = fval(ey);
        bool eopen = !eneg;
#pragma unroll
        for (int j = 0; j < KK; ++j) {
            const double yr = -(p2 * al[j] * be[j]) * rcp64_qp_nz(fma(p2 * al[j], al[j], pf));
            const double ej = fma(al[j], yr, be[j]);
            const bool cert = ej > 0.0 && ej >= emax(yr);
            const double y = fmin(fmax(yr, lo), hi);
            const double f = fval(y);
            const bool t = eopen && (cert || f < ef);
            ey = t ? y : ey;
            ef = t ? f : ef;
            eopen = eopen && !cert;
        }
        if (KK > 1 && __ballot(nd && eopen) != 0) {
#pragma unroll
            for (int i = 0; i < KK; ++i)
#pragma unroll
                for (int j = i + 1; j < KK; ++j) {
                    // den = 0: NaN, which the clamp turns into the feasible point lo
                    const double y = fmin(fmax((be[j] - be[i]) * rcp64_qp_nz(al[i] - al[j]), lo), hi);
                    const double f = fval(y);
                    const bool t = eopen && f < ef;
                    ey = t ? y : ey;
                    ef = t ? f : ef;
                }
        }
    };
    RCBF_QP_STAMP(1);
    bu0 = 0.0;
    bu1 = 0.0;
    bool all_neg = true;
#pragma unroll
    for (int j = 0; j < KK; ++j) all_neg = all_neg && (b[j] <= 0.0);
    bf = phi_e(0.0, 0.0, eps_of(0.0, 0.0));
    open = !all_neg;
    // stage 1a: the pieces' stationary points, with their certificates
#pragma unroll
    for (int j = 0; j < KK; ++j) {  // piece j: (diag(p0,p1) + p2 a a') u = -p2 b a
        double w0 = a0[j] * ip0, w1 = a1[j] * ip1;
        double sden = fma(p2, fma(a0[j], w0, a1[j] * w1), 1.0);
        double f = -p2 * b[j] * rcp64_qp_nz(sden);
        const double u0 = f * w0, u1 = f * w1;
        const double ej = fma(a0[j], u0, fma(a1[j], u1, b[j]));
        const double em = eps_of(u0, u1);
        const double fv = phi_e(u0, u1, em);
        const bool cert = ej > 0.0 && ej >= em;
        const bool t = open && (cert || fv < bf);
        bu0 = t ? u0 : bu0;
        bu1 = t ? u1 : bu1;
        bf = t ? fv : bf;
        open = open && !cert;
    }
    RCBF_QP_STAMP(2);
    RCBF_QP_COUNT(5, open);
    // stage 1b: kinks and triple points, for the uncertified lanes
    if (KK > 1 && __ballot(open) != 0) {
#pragma unroll
        for (int i = 0; i < KK; ++i) {
#pragma unroll
            for (int j = i + 1; j < KK; ++j) {  // kink line (a_i - a_j).u = b_j - b_i, minimise along it
                double d0 = a0[i] - a0[j], d1 = a1[i] - a1[j], c = b[j] - b[i];
                // parallel pieces (dd = 0) give NaN through rcp64_qp_nz and never win
                double dd = fma(d0, d0, d1 * d1);
                double idd = rcp64_qp_nz(dd);
                double q0 = c * d0 * idd, q1 = c * d1 * idd;  // a point on the line
                double n0 = -d1, n1 = d0;                     // its direction
                double ea = fma(a0[i], q0, fma(a1[i], q1, b[i])), an = fma(a0[i], n0, a1[i] * n1);
                double num = fma(p0 * q0, n0, fma(p1 * q1, n1, p2 * ea * an));
                double den = fma(p0 * n0, n0, fma(p1 * n1, n1, p2 * an * an));
                double t = -num * rcp64_qp_nz(den);
                take(fma(t, n0, q0), fma(t, n1, q1));
            }
        }
#pragma unroll
        for (int i = 0; i < KK; ++i) {
#pragma unroll
            for (int j = i + 1; j < KK; ++j) {
#pragma unroll
                for (int l = j + 1; l < KK; ++l) {  // triple point e_i = e_j = e_l
                    double m00 = a0[i] - a0[j], m01 = a1[i] - a1[j], r0 = b[j] - b[i];
                    double m10 = a0[i] - a0[l], m11 = a1[i] - a1[l], r1 = b[l] - b[i];
                    double det = fma(m00, m11, -m01 * m10);
                    double id = rcp64_qp_nz(det);  // det = 0: NaN, never wins
                    take((r0 * m11 - r1 * m01) * id, (m00 * r1 - m10 * r0) * id);
                }
            }
        }
    }
    const bool need0 = !((bu0 >= L0) && (bu0 <= U0)), need1 = !((bu1 >= L1) && (bu1 <= U1));
    const bool inbox = !need0 && !need1;
    RCBF_QP_STAMP(3);
    RCBF_QP_COUNT(6, need0);
    RCBF_QP_COUNT(7, need1);
    // stage 2: the facing u0-edge (u0 fixed, where u_f0 leaves [L0, U0]) and
    // u1-edge (where u_f1 leaves [L1, U1]), each only in waves with such a lane
    const double v0 = fmin(fmax(bu0, L0), U0), v1 = fmin(fmax(bu1, L1), U1);
    bf = inbox ? bf : __builtin_huge_val();  // an out-of-box stage-1 point must not win
    if (__ballot(need0) != 0) {
        double ey, ef;
        edge_solve(true, v0, L1, U1, need0, ey, ef);
        const bool t = need0 && ef < bf;
        bu0 = t ? v0 : bu0;
        bu1 = t ? ey : bu1;
        bf = t ? ef : bf;
    }
    RCBF_QP_STAMP(4);
    if (__ballot(need1) != 0) {
        double ey, ef;
        edge_solve(false, v1, L0, U0, need1, ey, ef);
        const bool t = need1 && ef < bf;
        bu0 = t ? ey : bu0;
        bu1 = t ? v1 : bu1;
        bf = t ? ef : bf;
    }
}

// Wave-uniform maximum of a small per-lane count (0..K).
template <int K>
__device__ __forceinline__ int wave_max_count(int cnt) {
    int kmax = 0;
#pragma unroll
    for (int t = 1; t <= K; ++t)
        if (__ballot(cnt >= t) != 0) kmax = t;
    return kmax;
}

// Slots 0..KK-1 of a lane: its first KK live rows in row order (mask bit j =
// row j live), compacted with selects (a lane-varying array index would be
// turned into LDS traffic by the compiler); slots past its live count repeat
// slot 0 (row 0 if none is live), which only adds NaN kink / triple
// candidates that never win.
template <int KK, int K, typename T>
__device__ __forceinline__ void uni_slots_solve(double p0, double p1, double p2, double ip0, double ip1,
                                                const T* a0, const T* a1, const T* b, unsigned mask, double L0,
                                                double U0, double L1, double U1, double& bu0, double& bu1,
                                                double& bf, double& e) {
    T S0[KK], S1[KK], SB[KK];
#pragma unroll
    for (int s = 0; s < KK; ++s) {
        S0[s] = a0[0];
        S1[s] = a1[0];
        SB[s] = b[0];
    }
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const bool live = (mask >> j) & 1u;
#pragma unroll
        for (int s = 0; s < KK && s <= j; ++s) {  // row j can only land in slots 0..j
            const bool here = live && (cnt == s);
            S0[s] = here ? a0[j] : S0[s];
            S1[s] = here ? a1[j] : S1[s];
            SB[s] = here ? b[j] : SB[s];
        }
        cnt += live ? 1 : 0;
    }
    double A0[KK], A1[KK], Bv[KK];
#pragma unroll
    for (int s = 0; s < KK; ++s) {  // unused slots repeat slot 0
        A0[s] = (double)((s == 0 || s < cnt) ? S0[s] : S0[0]);
        A1[s] = (double)((s == 0 || s < cnt) ? S1[s] : S1[0]);
        Bv[s] = (double)((s == 0 || s < cnt) ? SB[s] : SB[0]);
    }
    uni_pieces_solve<KK>(p0, p1, p2, ip0, ip1, A0, A1, Bv, L0, U0, L1, U1, bu0, bu1, bf);
    // eps at the optimum: the live rows' max (a dropped row has e_j <= 0 on the whole box)
    e = 0.0;
#pragma unroll
    for (int s = 0; s < KK; ++s) e = fmax(e, fma(A0[s], bu0, fma(A1[s], bu1, Bv[s])));
}

// The 2-D solve from the slack form: eps >= e_j(u) = a0_j u0 + a1_j u1 + b_j
// for the K hazard rows (T: float for the raw fp32 rows, double otherwise),
// the box [L0, U0] x [L1, U1]; finite: the caller's check of its inputs.
// Live rows (max over the box of e_j > 0; NaN data keeps the row, and such a
// lane fails below anyway) form a per-lane bit mask; the wave solves with KK
// = the largest live count of its lanes, picking only KK slots per lane.
template <int K, typename T>
__device__ __forceinline__ void uni_qp_2d_core(double p0, double p1, double p2, double ip0, double ip1,
                                               const T* a0, const T* a1, const T* b, double L0, double U0,
                                               double L1, double U1, bool finite, double* z, int& status) {
    RCBF_QP_STAMP(0);
    unsigned mask = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const double x0 = (double)a0[j], x1 = (double)a1[j];
        const double emax = (double)b[j] + fmax(x0 * L0, x0 * U0) + fmax(x1 * L1, x1 * U1);
        mask |= (emax <= 0.0 ? 0u : 1u) << j;
    }
    double bu0, bu1, bf, e;
    const int kmax = wave_max_count<K>(__popc(mask));
    RCBF_QP_COUNT(8, kmax > 0);
    RCBF_QP_COUNT(10, kmax > 1);
    RCBF_QP_COUNT(11, kmax > 2);
    if (kmax == 0) {  // no hazard row can bind anywhere in the box, for every lane of the wave
        bu0 = fmin(fmax(0.0, L0), U0);
        bu1 = fmin(fmax(0.0, L1), U1);
        bf = 0.0;
        e = 0.0;
    } else if (kmax == 1 || K == 1) {
        uni_slots_solve<1, K, T>(p0, p1, p2, ip0, ip1, a0, a1, b, mask, L0, U0, L1, U1, bu0, bu1, bf, e);
    } else if (kmax == 2 || K == 2) {
        uni_slots_solve<(K >= 2 ? 2 : 1), K, T>(p0, p1, p2, ip0, ip1, a0, a1, b, mask, L0, U0, L1, U1, bu0, bu1,
                                                bf, e);
    } else if (kmax == 3 || K == 3) {
        uni_slots_solve<(K >= 3 ? 3 : 1), K, T>(p0, p1, p2, ip0, ip1, a0, a1, b, mask, L0, U0, L1, U1, bu0, bu1,
                                                bf, e);
    } else {
        uni_slots_solve<K, K, T>(p0, p1, p2, ip0, ip1, a0, a1, b, mask, L0, U0, L1, U1, bu0, bu1, bf, e);
    }
    z[0] = bu0;
    z[1] = bu1;
    z[2] = e;
    RCBF_QP_STAMP(9);
    finite = finite && isfinite(U0 + L0 + U1 + L1);  // fmin/fmax would hide a NaN bound
    const bool ok = isfinite(z[0]) && isfinite(z[1]) && isfinite(z[2]) && bf < __builtin_huge_val();
    status = !finite ? RCBF_QP_NONFINITE : (ok && L0 <= U0 && L1 <= U1 ? RCBF_QP_OK : RCBF_QP_INFEASIBLE);
    if (!finite) z[0] = z[1] = z[2] = __builtin_nan("");
}

// uni_qp_2d_core's solve from a live-row mask computed elsewhere: the
// lane-pair STUDY build (csrc/study/rcbf_uni_pair.hip) forms the mask from the
// two lanes' halves of the hazard rows.  The product inlines uni_qp_2d_core
// (kept unchanged, so its machine code is untouched).
template <int K, typename T>
__device__ __forceinline__ void uni_qp_2d_masked(double p0, double p1, double p2, double ip0, double ip1,
                                                 const T* a0, const T* a1, const T* b, unsigned mask, double L0,
                                                 double U0, double L1, double U1, bool finite, double* z, int& status) {
    double bu0, bu1, bf, e;
    const int kmax = wave_max_count<K>(__popc(mask));
    RCBF_QP_COUNT(8, kmax > 0);
    RCBF_QP_COUNT(10, kmax > 1);
    RCBF_QP_COUNT(11, kmax > 2);
    if (kmax == 0) {  // no hazard row can bind anywhere in the box, for every lane of the wave
        bu0 = fmin(fmax(0.0, L0), U0);
        bu1 = fmin(fmax(0.0, L1), U1);
        bf = 0.0;
        e = 0.0;
    } else if (kmax == 1 || K == 1) {
        uni_slots_solve<1, K, T>(p0, p1, p2, ip0, ip1, a0, a1, b, mask, L0, U0, L1, U1, bu0, bu1, bf, e);
    } else if (kmax == 2 || K == 2) {
        uni_slots_solve<(K >= 2 ? 2 : 1), K, T>(p0, p1, p2, ip0, ip1, a0, a1, b, mask, L0, U0, L1, U1, bu0, bu1,
                                                bf, e);
    } else if (kmax == 3 || K == 3) {
        uni_slots_solve<(K >= 3 ? 3 : 1), K, T>(p0, p1, p2, ip0, ip1, a0, a1, b, mask, L0, U0, L1, U1, bu0, bu1,
                                                bf, e);
    } else {
        uni_slots_solve<K, K, T>(p0, p1, p2, ip0, ip1, a0, a1, b, mask, L0, U0, L1, U1, bu0, bu1, bf, e);
    }
    z[0] = bu0;
    z[1] = bu1;
    z[2] = e;
    RCBF_QP_STAMP(9);
    finite = finite && isfinite(U0 + L0 + U1 + L1);  // fmin/fmax would hide a NaN bound
    const bool ok = isfinite(z[0]) && isfinite(z[1]) && isfinite(z[2]) && bf < __builtin_huge_val();
    status = !finite ? RCBF_QP_NONFINITE : (ok && L0 <= U0 && L1 <= U1 ? RCBF_QP_OK : RCBF_QP_INFEASIBLE);
    if (!finite) z[0] = z[1] = z[2] = __builtin_nan("");
}


// On the normalised rows (what qpth sees): back to the slack form by one
// division per row by its (negative) slack coefficient.
template <int K, typename R>
__device__ __forceinline__ void uni_qp_2d(const PMat<3, true>& pm, const R (*G)[3], const R* h, double* z,
                                          int& status) {
    double a0[K], a1[K], b[K];
    bool finite = true;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const double inv = rcp64_qp_nz((double)G[j][2]);
        a0[j] = -(double)G[j][0] * inv;
        a1[j] = -(double)G[j][1] * inv;
        b[j] = (double)h[j] * inv;
        finite = finite && isfinite(a0[j]) && isfinite(a1[j]) && isfinite(b[j]);
    }
    const double U0 = (double)h[K] * rcp64_qp_nz((double)G[K][0]);
    const double L0 = (double)h[K + 1] * rcp64_qp_nz((double)G[K + 1][0]);
    const double U1 = (double)h[K + 2] * rcp64_qp_nz((double)G[K + 2][1]);
    const double L1 = (double)h[K + 3] * rcp64_qp_nz((double)G[K + 3][1]);
    uni_qp_2d_core<K, double>(pm.P[0][0], pm.P[1][1], pm.P[2][2], pm.Pinv[0][0], pm.Pinv[1][1], a0, a1, b, L0, U0,
                              L1, U1, finite, z, status);
}

// On the RAW rows (the fused safe step; see cars_qp_1d_raw for why the
// normalisation can be skipped): hazard rows -a_j.u - eps <= h_j have slack
// coefficient -1 exactly (uni_rows_diff_cs), so e_j(u) = G_j0 u0 + G_j1 u1
// - h_j with the fp32 entries as they are, and the actuator rows are +-1:
// U0 = h_K, L0 = -h_{K+1}, U1 = h_{K+2}, L1 = -h_{K+3}.  No division at all.
template <int K, typename R>
__device__ __forceinline__ void uni_qp_2d_raw(const PMat<3, true>& pm, const R (*G)[3], const R* h, double* z,
                                              int& status) {
    R a0[K], a1[K], b[K];
    double chk = 0.0;  // NaN / inf in any entry makes the sum non-finite (fp32 inputs cannot overflow it)
#pragma unroll
    for (int j = 0; j < K; ++j) {
        a0[j] = G[j][0];
        a1[j] = G[j][1];
        b[j] = -h[j];  // exact
        chk += ((double)a0[j] + (double)a1[j]) + ((double)b[j] + (double)G[j][2]);
    }
    const double U0 = (double)h[K], L0 = -(double)h[K + 1];
    const double U1 = (double)h[K + 2], L1 = -(double)h[K + 3];
    uni_qp_2d_core<K, R>(pm.P[0][0], pm.P[1][1], pm.P[2][2], pm.Pinv[0][0], pm.Pinv[1][1], a0, a1, b, L0, U0, L1,
                         U1, isfinite(chk), z, status);
}

// Compile-time solver choice (the host dispatches on rcbf_params.solver):
//   RCBF_SOLVER_ACTIVE_SET: exact -- KKT enumeration for n = 2, Goldfarb-Idnani
//                           for n = 3 or a full P;
//   RCBF_SOLVER_GI:         Goldfarb-Idnani for every size;
//   RCBF_SOLVER_PDIPM:      primal-dual interior point + active-set polish.
template <int SOLVER, int N, int M, bool DIAG, typename R>
__device__ __forceinline__ void qp_solve(const PMat<N, DIAG>& pm, const double* q, const R (*G)[N],
                                         const R* h, int max_iter, double eps, QPResult<N, M>& out) {
    if constexpr (SOLVER == RCBF_SOLVER_PDIPM) {
        pdipm_solve<N, M, DIAG, R>(pm, q, G, h, max_iter > 0 ? max_iter : 50, eps > 0 ? eps : 1e-10, out);
        // qpth returns its best iterate when it stalls (notImprovedLim), which
        // can be far from the optimum on badly scaled rows; a point that fails
        // the KKT certificate is re-solved exactly instead (rare lanes only).
        if (!out.certified && out.status != RCBF_QP_NONFINITE) {
            const int its = out.iters;
            gi_solve<N, M, DIAG, R>(pm, q, G, h, 4 * (M + N) + 8, out);
            out.iters = its;
        }
    } else if constexpr (SOLVER == RCBF_SOLVER_ACTIVE_SET && N == 2 && DIAG) {
        enum2_solve_fast<M, R>(pm, G, h, out);
    } else {
        gi_solve<N, M, DIAG, R>(pm, q, G, h, max_iter > 0 ? max_iter : 4 * (M + N) + 8, out);
    }
}

// ---------------------------------------------------------------------------
// Row normalisation  (diff_cbf_qp.py:103-106 / cbf_qp.py:270-273)
//   N_r = max(|G_r|_inf, |h_r|);  G_r /= N_r;  h_r /= N_r
// argmax_is_h records whether torch.max picked the h entry (first maximum
// wins, as torch.max(dim) returns the first maximal index) -- the backward
// routes dN/dh only through that entry.
// ---------------------------------------------------------------------------
template <int N, int M, typename T>
__device__ __forceinline__ void normalize_rows(T (*G)[N], T* h, T* Nrm, bool* argmax_is_h, double* rinv = nullptr) {
#pragma unroll
    for (int r = 0; r < M; ++r) {
        T mx = fabs(G[r][0]);
#pragma unroll
        for (int k = 1; k < N; ++k) mx = fmax(mx, fabs(G[r][k]));
        T ah = fabs(h[r]);
        bool ish = ah > mx;
        T nr = ish ? ah : mx;
        Nrm[r] = nr;
        if (argmax_is_h) argmax_is_h[r] = ish;
        if constexpr (sizeof(T) == 4) {
            // one reciprocal per row, exact fp32 quotients; nr = 0 only for an
            // all-zero row, whose quotients are NaN either way (0 * inf, 0 * NaN)
            const double rn = rcp64_nz((double)nr);
            if (rinv) rinv[r] = rn;
#pragma unroll
            for (int k = 0; k < N; ++k) G[r][k] = div_f32_via_rcp(G[r][k], rn);
            h[r] = div_f32_via_rcp(h[r], rn);
        } else {
#pragma unroll
            for (int k = 0; k < N; ++k) G[r][k] = G[r][k] / nr;
            h[r] = h[r] / nr;
        }
    }
}

// The same normalisation for the layer's rows, knowing their structure: the
// last 2 n_u rows are the actuator box (one +-1 entry, zeros elsewhere,
// diff_cbf_qp.py:362-377), so N = max(1, |h|), the unit entry becomes
// +-RN32(1/N), the zeros stay +0 (0 / N for finite N >= 1) and h becomes
// RN32(h / N) -- the values normalize_rows produces, without the zero
// entries' arithmetic.  The CBF rows take the general path.
template <int N, int M, int NBOX>
__device__ __forceinline__ void normalize_layer_rows(float (*G)[N], float* h, float* Nrm, bool* argmax_is_h) {
    normalize_rows<N, M - NBOX, float>(G, h, Nrm, argmax_is_h);
#pragma unroll
    for (int r = M - NBOX; r < M; ++r) {
        const int c = (r - (M - NBOX)) >> 1;  // the bounded coordinate
        const float g = G[r][c];              // +-1
        const float ah = fabsf(h[r]);
        const bool ish = ah > fabsf(g);
        const float nr = ish ? ah : fabsf(g);
        Nrm[r] = nr;
        if (argmax_is_h) argmax_is_h[r] = ish;
        const double rn = rcp64_nz((double)nr);
#pragma unroll
        for (int k = 0; k < N; ++k) G[r][k] = (k == c) ? div_f32_via_rcp(g, rn) : 0.0f;
        h[r] = div_f32_via_rcp(h[r], rn);
    }
}

// ---------------------------------------------------------------------------
// CBF constraint builders
// ---------------------------------------------------------------------------
// SimulatedCars, CBFQPLayer form (diff_cbf_qp.py:268-357, actuators 362-377).
// fp32, torch's elementwise order; mu is not used by the reference.
// sig5/7/9 = sigma[:, 5], [:, 7], [:, 9] (fD_x at the odd entries, :298-299).
__device__ __forceinline__ void cars_rows_diff(const rcbf_params& prm, const float* xs, float u,
                                               float sig5, float sig7, float sig9, float (*G)[2],
                                               float* h) {
#pragma clang fp contract(off)
    const float kp = (float)prm.kp, kb = (float)prm.k_brake;
    float p0 = xs[0], p1 = xs[2], p2 = xs[4], p3 = xs[6], p4 = xs[8];
    float v0 = xs[1], v1 = xs[3], v2 = xs[5], v3 = xs[7], v4 = xs[9];
    (void)v0;
    float a1 = kp * (30.0f - v1), a2 = kp * (30.0f - v2), a4 = kp * (30.0f - v4);
    float d01 = p0 - p1, d12 = p1 - p2, d24 = p2 - p4;
    a1 = a1 - (kb * d01) * (d01 < 6.0f ? 1.0f : 0.0f);
    a2 = a2 - (kb * d12) * (d12 < 6.0f ? 1.0f : 0.0f);
    const float a3 = 0.0f;  // car 4's acceleration is the control (:289)
    a4 = a4 - (kb * d24) * (d24 < 13.0f ? 1.0f : 0.0f);
    float e23 = p2 - p3, e43 = p4 - p3;
    float h13 = 0.5f * ((e23 * e23) - 12.25f);
    float h15 = 0.5f * ((e43 * e43) - 12.25f);
    float h13d = (p3 - p2) * (v3 - v2);
    float h15d = (p3 - p4) * (v3 - v4);
    float c4 = v2 - v3, c5 = p2 - p3, c6 = v3 - v2, c7 = p3 - p2;
    float Lff13 = ((c4 * v2 + c5 * a2) + c6 * v3) + c7 * a3;
    float LfD13 = fabsf(c5) * sig5 + fabsf(c7) * sig7;
    float e6 = v3 - v4, e7 = p3 - p4, e8 = v4 - v3, e9 = p4 - p3;
    float Lff15 = ((e6 * v3 + e7 * a3) + e8 * v4) + e9 * a4;
    float LfD15 = fabsf(e7) * sig7 + fabsf(e9) * sig9;
    float Lg13 = c7 * 50.0f, Lg15 = e7 * 50.0f;
    const float gg = (float)(prm.gamma_b + prm.gamma_b);
    const float g2 = (float)(prm.gamma_b * prm.gamma_b);
    h[0] = (((Lff13 - LfD13) + gg * h13d) + g2 * h13) + Lg13 * u;
    h[1] = (((Lff15 - LfD15) + gg * h15d) + g2 * h15) + Lg15 * u;
    G[0][0] = -Lg13;
    G[0][1] = -200.0f;
    G[1][0] = -Lg15;
    G[1][1] = -200.0f;
    G[2][0] = 1.0f;
    G[2][1] = 0.0f;
    h[2] = (float)prm.u_max[0] - u;
    G[3][0] = -1.0f;
    G[3][1] = 0.0f;
    h[3] = -(float)prm.u_min[0] + u;
}

// SimulatedCars, CascadeCBFLayer form (cbf_qp.py:149-219), fp64: no robust
// term, mean/sigma ignored (:210-211).
__device__ __forceinline__ void cars_rows_cascade(const rcbf_params& prm, const double* xs, double u,
                                                  double (*G)[2], double* h) {
#pragma clang fp contract(off)
    const double kp = prm.kp, kb = prm.k_brake, g = prm.gamma_b;
    double p0 = xs[0], p1 = xs[2], p2 = xs[4], p3 = xs[6], p4 = xs[8];
    double v1 = xs[3], v2 = xs[5], v3 = xs[7], v4 = xs[9];
    double a2 = kp * (30.0 - v2), a4 = kp * (30.0 - v4);
    double d01 = p0 - p1, d12 = p1 - p2, d24 = p2 - p4;
    (void)d01;
    (void)v1;
    a2 = a2 - kb * d12 * (d12 < 6.0 ? 1.0 : 0.0);
    a4 = a4 - kb * d24 * (d24 < 13.0 ? 1.0 : 0.0);
    const double a3 = 0.0;
    double h13 = 0.5 * ((p2 - p3) * (p2 - p3) - 12.25);
    double h15 = 0.5 * ((p4 - p3) * (p4 - p3) - 12.25);
    double h13d = (p3 - p2) * (v3 - v2);
    double h15d = (p3 - p4) * (v3 - v4);
    double Lff13 = (((v2 - v3) * v2 + (p2 - p3) * a2) + (v3 - v2) * v3) + (p3 - p2) * a3;
    double Lff15 = (((v3 - v4) * v3 + (p3 - p4) * a3) + (v4 - v3) * v4) + (p4 - p3) * a4;
    double Lg13 = (p3 - p2) * 50.0, Lg15 = (p3 - p4) * 50.0;
    h[0] = ((Lff13 + (g + g) * h13d) + g * g * h13) + Lg13 * u;
    h[1] = ((Lff15 + (g + g) * h15d) + g * g * h15) + Lg15 * u;
    G[0][0] = -Lg13;
    G[0][1] = -2e2;
    G[1][0] = -Lg15;
    G[1][1] = -2e2;
    G[2][0] = 1.0;
    G[2][1] = 0.0;
    h[2] = prm.u_max[0] - u;
    G[3][0] = -1.0;
    G[3][1] = 0.0;
    h[3] = -prm.u_min[0] + u;
}

// Unicycle, CBFQPLayer form (diff_cbf_qp.py:202-266, actuators 362-377), fp32.
// K hazards -> rows 0..K-1; actuator rows K..K+3 in the reference's order.
// rows from c = fp32 cos(theta32), s = fp32 sin(theta32) (theta32 = xs[2])
template <int K>
__device__ __forceinline__ void uni_rows_diff_cs(const rcbf_params& prm, const float* xs, float c, float s,
                                                 const float* u, const float* mu, const float* sig,
                                                 float (*G)[3], float* h) {
#pragma clang fp contract(off)
    const float lp = (float)prm.l_p, g = (float)prm.gamma_b;
    float px = xs[0] + lp * c, py = xs[1] + lp * s;
    float g00 = c, g01 = -s * lp, g10 = s, g11 = c * lp;
    float mupx = g01 * mu[2] + mu[0], mupy = g11 * mu[2] + mu[1];
    float sgpx = fabsf(g01) * sig[2] + sig[0], sgpy = fabsf(g11) * sig[2] + sig[1];
    const float r2 = (float)((1.2 * prm.hazards_radius) * (1.2 * prm.hazards_radius));
#pragma unroll
    for (int j = 0; j < K; ++j) {
        float ox = (float)prm.hazards_xy[2 * j], oy = (float)prm.hazards_xy[2 * j + 1];
        float dx = px - ox, dy = py - oy;
        float hs = 0.5f * ((dx * dx + dy * dy) - r2);
        float a0 = dx * g00 + dy * g10;
        float a1 = dx * g01 + dy * g11;
        float t1 = dx * mupx + dy * mupy;
        float t2 = fabsf(dx) * sgpx + fabsf(dy) * sgpy;
        float t3 = a0 * u[0] + a1 * u[1];
        G[j][0] = -a0;
        G[j][1] = -a1;
        G[j][2] = -1.0f;
        h[j] = g * ((hs * hs) * hs) + ((t1 - t2) + t3);
    }
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
        const int r0 = K + 2 * c2;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            G[r0][k] = (k == c2) ? 1.0f : 0.0f;
            G[r0 + 1][k] = (k == c2) ? -1.0f : 0.0f;
        }
        h[r0] = (float)prm.u_max[c2] - u[c2];
        h[r0 + 1] = -(float)prm.u_min[c2] + u[c2];
    }
}

template <int K>
__device__ __forceinline__ void uni_rows_diff(const rcbf_params& prm, const float* xs, const float* u,
                                              const float* mu, const float* sig, float (*G)[3], float* h) {
    // fp32 cos/sin, correctly rounded from fp64 (torch's SLEEF is within 1 ulp)
    double sd, cd;
    sincos((double)xs[2], &sd, &cd);  // one shared range reduction
    uni_rows_diff_cs<K>(prm, xs, (float)cd, (float)sd, u, mu, sig, G, h);
}

// get_state(float(obs(x))) of a unicycle state whose cos/sin c, s (fp64) are
// already known, plus the fp32 cos/sin of the resulting theta32 that the rows
// need -- without the atan2 and the second sincos.
//   obs[2:4] = (c32, s32) = RN32(c, s);  the reference's theta32 =
//   RN32(atan2(s32, c32)) (dynamics.py:205-232, fp64 arctan2 then fp32).
//   With ds = s32 - s, dc = c32 - c (exact, Sterbenz): atan2(s32, c32) =
//   t + (c ds - s dc) / (c^2 + s^2) + O(|d|^2 ~ 4e-15), t = theta reduced to
//   (-pi, pi] (two-constant Cody-Waite), wrapped to the side atan2 returns
//   (the sign of s32).  Then cos/sin(theta32) = cos/sin(t + D) with
//   D = theta32 - t' (|D| <~ 1e-7) by the addition formulas.  Both results
//   are RN32 of a value within ~1e-15 of the exact one, i.e. the reference's
//   value except within ~1e-15 of an fp32 rounding midpoint (a 1-ulp
//   difference there; tests/test_solver_math.py test_uni_theta32_from_cos_sin).
__device__ __forceinline__ void uni_state32_from_cs(const double* xs, double c, double s, float* s32, float& c_row,
                                                    float& s_row) {
    const double kPi = 3.141592653589793116, k2PiHi = 6.28318530717958623200, k2PiLo = 2.44929359829470635e-16;
    const float c32 = (float)c, s32f = (float)s;
    const double dc = (double)c32 - c, ds = (double)s32f - s;
    const double k = rint(xs[2] * (1.0 / k2PiHi));
    double t0 = fma(-k, k2PiLo, fma(-k, k2PiHi, xs[2]));  // the angle of (c, s), up to ~1e-16 k
    // the angle of (c32, s32): t0 + (c ds - s dc) / (c^2 + s^2), where c^2 + s^2 = 1 within a few ulps,
    // so dividing the ~1e-8 correction by it would change t by ~1e-24 -- it is left out
    double t = t0 + fma(c, ds, -s * dc);
    const double wrap = (s32f > 0.0f && t < 0.0) ? k2PiHi : ((s32f < 0.0f && t > 0.0) ? -k2PiHi : 0.0);
    t += wrap;
    t0 += wrap;
    // exact zeros of s32: atan2(+-0, c32 > 0) = +-0, atan2(+-0, c32 < 0) = +-pi (then |s| < 1e-45:
    // the true angle is that value)
    const double tz = c32 < 0.0f ? __builtin_copysign(kPi, (double)s32f) : __builtin_copysign(0.0, (double)s32f);
    t = (s32f == 0.0f) ? tz : t;
    t0 = (s32f == 0.0f) ? tz : t0;
    const float th32 = (float)t;
    s32[0] = (float)xs[0];
    s32[1] = (float)xs[1];
    s32[2] = th32;
    // cos/sin(theta32) = cos/sin(t0 + D) with (c, s) = cos/sin(t0), D = theta32 - t0 (|D| <~ 2e-7)
    const double D = (double)th32 - t0;
    const double D2 = D * D;
    const double cD = fma(D2, fma(D2, 1.0 / 24.0, -0.5), 1.0), sD = D * fma(D2, -1.0 / 6.0, 1.0);
    c_row = (float)fma(c, cD, -(s * sD));
    s_row = (float)fma(s, cD, c * sD);
}

// Unicycle, CascadeCBFLayer form (cbf_qp.py:91-147), fp64: signed sigma_p,
// robust term x k_d.
template <int K>
__device__ __forceinline__ void uni_rows_cascade(const rcbf_params& prm, const double* xs, const double* u,
                                                 const double* mu, const double* sig, double (*G)[3],
                                                 double* h) {
#pragma clang fp contract(off)
    const double lp = prm.l_p, g = prm.gamma_b, kd = prm.k_d;
    double c, s;
    sincos(xs[2], &s, &c);
    double px = xs[0] + lp * c, py = xs[1] + lp * s;
    double g00 = c, g01 = -s * lp, g10 = s, g11 = c * lp;
    double mpx = mu[0] + lp * (-s) * mu[2], mpy = mu[1] + lp * c * mu[2];
    double spx = sig[0] + lp * (-s) * sig[2], spy = sig[1] + lp * c * sig[2];
    const double r2 = (1.2 * prm.hazards_radius) * (1.2 * prm.hazards_radius);
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double dx = px - prm.hazards_xy[2 * j], dy = py - prm.hazards_xy[2 * j + 1];
        double hs = 0.5 * ((dx * dx + dy * dy) - r2);
        double a0 = dx * g00 + dy * g10, a1 = dx * g01 + dy * g11;
        G[j][0] = -a0;
        G[j][1] = -a1;
        G[j][2] = -1.0;
        h[j] = ((g * (hs * hs * hs) + (dx * mpx + dy * mpy)) + (a0 * u[0] + a1 * u[1])) -
               kd * (fabs(dx) * spx + fabs(dy) * spy);
    }
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
        const int r0 = K + 2 * c2;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            G[r0][k] = (k == c2) ? 1.0 : 0.0;
            G[r0 + 1][k] = (k == c2) ? -1.0 : 0.0;
        }
        h[r0] = prm.u_max[c2] - u[c2];
        h[r0 + 1] = -prm.u_min[c2] + u[c2];
    }
}

// ---------------------------------------------------------------------------
// environments (fp64, numpy order, no contraction)
// ---------------------------------------------------------------------------
struct CarsStepOut {
    float reward;
    double reward_d;
    double cost;
    bool done;
};

// SimulatedCarsEnv.step (simulated_cars_env.py:38-106): true dynamics with
// the lead car's sin term, car 4's kp drift kept, x1.1 on every acceleration,
// split at the safe action: cars_env_pre is everything
// that does not depend on it (all positions, the velocities of cars 0, 1, 2
// and 4, t, step, done, cost) and returns car 3's acceleration; cars_env_post
// adds g u to car 3's velocity and forms the reward.  pre + post is exactly
// the reference's step.  k_safe_step stores the state the pre part fixes
// before the layer's chain runs (RCBF_EARLY_STORE, the product default since
// r03: 3.85 -> 3.67 us per step, profiles/r03/early_store_confirm_r03k.txt;
// r01's first form of it measured no faster, profiles/r01/ablate_early_store.txt).
__device__ __forceinline__ double cars_env_pre(const rcbf_params& prm, double* xs, double& t, int& step,
                                               CarsStepOut& o) {
#pragma clang fp contract(off)
    const double kp = prm.kp, kb = prm.k_brake, dt = 0.02;
    double vdes0 = 30.0 - 10.0 * sin_small(0.2 * t);
    double acc[5];
    acc[0] = kp * (vdes0 - xs[1]);
#pragma unroll
    for (int i = 1; i < 5; ++i) acc[i] = kp * (30.0 - xs[2 * i + 1]);
    double d01 = xs[0] - xs[2], d12 = xs[2] - xs[4], d24 = xs[4] - xs[8];
    acc[1] += (-kb * d01) * (d01 < 6.0 ? 1.0 : 0.0);
    acc[2] += (-kb * d12) * (d12 < 6.0 ? 1.0 : 0.0);
    acc[4] += (-kb * d24) * (d24 < 13.0 ? 1.0 : 0.0);
#pragma unroll
    for (int i = 0; i < 5; ++i) acc[i] *= 1.1;
    double v[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) v[i] = xs[2 * i + 1];
    // x += dt * (f + g u): the reference adds g u = 0.0 to every component but
    // car 3's velocity; v + 0.0 differs from v only for v = -0.0, and then only
    // in the sign of a zero, so those adds are skipped.
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        xs[2 * i] += dt * v[i];
        if (i != 3) xs[2 * i + 1] += dt * acc[i];
    }
    t = t + dt;
    step += 1;
    o.done = step >= 300;
    double cost = 0.0;
    if (xs[4] - xs[6] < 2.99) cost -= 0.1;
    if (xs[6] - xs[8] < 2.99) cost -= 0.1;
    o.cost = cost;
    return acc[3];
}

template <typename A>
__device__ __forceinline__ void cars_env_post(double* xs, double acc3, A action, CarsStepOut& o) {
#pragma clang fp contract(off)
    const double dt = 0.02;
    const double gu = 50.0 * (double)action;
    xs[7] += dt * (acc3 + gu);
    // reward in the action's dtype (-5.0 * abs(a**2) / 300), :93
    A a2 = action * action;
    A r = (A)(-5.0) * (a2 < (A)0 ? -a2 : a2) / (A)300;
    o.reward = (float)r;
    o.reward_d = (double)r;
}

// SimulatedCarsEnv.step (simulated_cars_env.py:38-106)
template <typename A>
__device__ __forceinline__ void cars_env_step(const rcbf_params& prm, double* xs, double& t, int& step, A action,
                                              CarsStepOut& o) {
    const double acc3 = cars_env_pre(prm, xs, t, step, o);
    cars_env_post<A>(xs, acc3, action, o);
}

// x / d for a constant d, correctly rounded: q = RN(x * RN(1/d)) is within
// 1 ulp of x/d, r = x - q*d is exact with one FMA, and q + r*RN(1/d) rounds
// to RN(x/d) (Markstein's theorem).  3 FMA-pipe ops instead of the ~10-op
// v_div_scale/v_rcp/v_div_fmas/v_div_fixup sequence of a general division.
__device__ __forceinline__ double div_const(double x, double d, double inv_d) {
    double q = x * inv_d;
    double r = fma(-q, d, x);
    return fma(r, inv_d, q);
}

__device__ __forceinline__ void cars_obs(const double* xs, double* o) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        o[2 * i] = div_const(xs[2 * i], 100.0, 1.0 / 100.0);       // obs[::2] /= 100 (:156)
        o[2 * i + 1] = div_const(xs[2 * i + 1], 30.0, 1.0 / 30.0);  // obs[1::2] /= 30 (:157)
    }
}

// cos/sin of (theta + d) from c = cos theta, s = sin theta, |d| <= 0.05:
// Taylor to d^9 / d^8 (truncation < 1e-19), then the addition formulas;
// a couple of ulps from cos/sin(theta + d) evaluated directly.
__device__ __forceinline__ void sincos_add_small(double c, double s, double d, double& c2, double& s2) {
    const double d2 = d * d;
    const double sd =
        d * fma(d2, fma(d2, fma(d2, fma(d2, 1.0 / 362880.0, -1.0 / 5040.0), 1.0 / 120.0), -1.0 / 6.0), 1.0);
    const double cd =
        fma(d2, fma(d2, fma(d2, fma(d2, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5), 1.0);
    c2 = fma(c, cd, -(s * sd));
    s2 = fma(s, cd, c * sd);
}

__device__ __forceinline__ double uni_goal_dist(const double* xs) {
#pragma clang fp contract(off)
    double d0 = 2.5 - xs[0], d1 = 2.5 - xs[1];
    return sqrt(d0 * d0 + d1 * d1);
}

// UnicycleEnv.get_obs (unicycle_env.py:215-231) + obs_compass (:260-277)
// obs from precomputed cos/sin of theta and goal distance (the env step
// already has them for the new state)
__device__ __forceinline__ void uni_obs_cs(const double* xs, double c, double s, double gd, double* o) {
#pragma clang fp contract(off)
    double r0 = 2.5 - xs[0], r1 = 2.5 - xs[1];
    double v0 = r0 * c + r1 * s;
    double v1 = r0 * (-s) + r1 * c;
    double nrm = sqrt(v0 * v0 + v1 * v1) + 0.001;
    // the fused step stores these as fp32: one reciprocal (within an ulp of
    // the fp64 quotient, so the same fp32 value but at an fp32 rounding midpoint)
    const double rn = rcp64_nz(nrm);
    o[0] = xs[0];
    o[1] = xs[1];
    o[2] = c;
    o[3] = s;
    o[4] = v0 * rn;
    o[5] = v1 * rn;
    o[6] = exp(-gd);
}

__device__ __forceinline__ void uni_obs(const double* xs, double* o) {
#pragma clang fp contract(off)
    double r0 = 2.5 - xs[0], r1 = 2.5 - xs[1];
    double gd = sqrt(r0 * r0 + r1 * r1);
    double c, s;
    sincos(xs[2], &s, &c);
    double v0 = r0 * c + r1 * s;
    double v1 = r0 * (-s) + r1 * c;
    double nrm = sqrt(v0 * v0 + v1 * v1) + 0.001;
    o[0] = xs[0];
    o[1] = xs[1];
    o[2] = c;
    o[3] = s;
    o[4] = v0 / nrm;
    o[5] = v1 / nrm;
    o[6] = exp(-gd);
}

struct UniStepOut {
    double reward;
    double cost;
    bool done;
    bool goal;
    double c, s, gd;  // cos/sin of the new theta and the new goal distance (for the obs)
};

// UnicycleEnv.step/_step (unicycle_env.py:46-111): clip to +-1 after the
// safety filter, Euler step with g(x), then the -(dt*0.1) g(x') [cos th', 0]
// drift evaluated left to right (:87).
// KH > 0: the hazard count known at compile time (the fused step; the cost
// test unrolls and reuses the hazard positions the rows already loaded,
// instead of a loop of dependent scalar loads); 0: prm.num_hazards.
template <typename A, int KH = 0>
__device__ __forceinline__ void uni_env_step_cs(const rcbf_params& prm, double* xs, double& last_dist, int& step,
                                                const A* action, double c, double s, UniStepOut& o) {
#pragma clang fp contract(off)
    A a0c = action[0] < (A)(-1) ? (A)(-1) : (action[0] > (A)1 ? (A)1 : action[0]);
    A a1c = action[1] < (A)(-1) ? (A)(-1) : (action[1] > (A)1 ? (A)1 : action[1]);
    double a0 = (double)a0c, a1 = (double)a1c;
    const double dt = 0.02;
    // f = 0: 0.0 + g u equals g u up to the sign of a zero (skipped)
    xs[0] += dt * (c * a0);
    xs[1] += dt * (s * a0);
    const double th0 = xs[2];
    xs[2] += dt * a1;
    // cos/sin of the new theta by angle addition from the old one (|delta| <= 0.02)
    double c2, s2;
    sincos_add_small(c, s, xs[2] - th0, c2, s2);
    const double k = dt * 0.1;
    xs[0] -= (k * c2) * c2;
    xs[1] -= (k * s2) * c2;
    o.c = c2;
    o.s = s2;
    step += 1;
    double d = uni_goal_dist(xs);
    o.gd = d;
    double reward = last_dist - d;
    last_dist = d;
    bool goal = d <= 0.3;
    if (goal) reward += 1.0;
    o.goal = goal;
    o.done = goal || (step >= 1000);
    o.reward = reward;
    bool hit = false;
    const double r2 = prm.hazards_radius * prm.hazards_radius;
    const int nh = KH > 0 ? KH : prm.num_hazards;
#pragma unroll
    for (int j = 0; j < nh; ++j) {
        double ex = xs[0] - prm.hazards_xy[2 * j], ey = xs[1] - prm.hazards_xy[2 * j + 1];
        hit = hit || (ex * ex + ey * ey < r2);
    }
    o.cost = hit ? 0.1 : 0.0;
}

template <typename A>
__device__ __forceinline__ void uni_env_step(const rcbf_params& prm, double* xs, double& last_dist, int& step,
                                             const A* action, UniStepOut& o) {
    double c, s;
    sincos(xs[2], &s, &c);
    uni_env_step_cs<A>(prm, xs, last_dist, step, action, c, s, o);
}

// ---------------------------------------------------------------------------
// counter-based RNG (Philox4x32-10) for the cars reset draw N(0, 0.5)
// keyed by (seed, global env index, episode counter) -> independent of how
// envs are sharded over GPUs.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one v_mad_u64_u32 per 32 x 32 -> 64 product (hi and lo together)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// Reset draw: Box-Muller on 24-bit uniforms with the hardware fp32
// log2/cos -- ~10 instructions instead of ~170 for an fp64 libm path; the
// reset branch is on the critical path of whichever wave holds a resetting
// env, and this took the cars step at SURVEY start states from 5.3 to 4.9 us
// (profiles/r01).  Statistically a N(0,1) draw (|z| <= 5.8 with 24-bit
// uniforms); restated by oracle.normal_draw.
__device__ __forceinline__ double normal_draw(uint64_t seed, uint64_t env, uint32_t episode) {
    uint32_t c[4] = {(uint32_t)env, (uint32_t)(env >> 32), episode, 0x5AFEu};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    // hardware fp32 transcendentals (v_log_f32, v_cos_f32 takes revolutions)
    float f1 = ((float)(c[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);
    float f2 = (float)(c[2] >> 8) * (1.0f / 16777216.0f);
    return (double)(__builtin_sqrtf(-2.0f * __builtin_amdgcn_logf(f1) * 0.69314718f) * __builtin_amdgcn_cosf(f2));
}

__device__ __forceinline__ void cars_reset_state(double* xs, double noise) {
    const double p0[5] = {34.0, 28.0, 22.0, 16.0, 10.0};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        xs[2 * i] = p0[i];
        xs[2 * i + 1] = 30.0 + noise;
    }
    xs[7] = 35.0;
}

__device__ __forceinline__ void uni_reset_state(double* xs, double& last_dist) {
    xs[0] = -2.5;
    xs[1] = -2.5;
    xs[2] = 0.0;
    last_dist = uni_goal_dist(xs);
}

}  // namespace rcbf
