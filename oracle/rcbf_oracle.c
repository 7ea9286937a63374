/*
 * rcbf_oracle.c -- CPU ORACLE, TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the batched safe-env step of SAC-RCBF, used by
 * tests/ as a second checker and by bench.py's cpu_baseline leg (OpenMP over
 * envs).  Never linked into or called by the product path.  Same algorithm
 * and arithmetic as oracle/oracle.py (pinned against tests/golden/*.npz):
 *
 *   CBFQPLayer rows, SimulatedCars   rcbf_sac/diff_cbf_qp.py:268-357,362-377 (fp32)
 *   CBFQPLayer rows, Unicycle        rcbf_sac/diff_cbf_qp.py:202-266,362-377 (fp32)
 *   row normaliser                   rcbf_sac/diff_cbf_qp.py:103-106          (fp32)
 *   QP (qpth/quadprog, absent)       exact optimum by active-set enumeration  (fp64)
 *   clamp(u_RL + u_qp)               rcbf_sac/diff_cbf_qp.py:77               (fp32)
 *   SimulatedCarsEnv.step            envs/simulated_cars_env.py:38-106        (fp64)
 *   UnicycleEnv.step                 envs/unicycle_env.py:46-111              (fp64)
 *   get_state(obs32)                 rcbf_sac/dynamics.py:190-232
 *
 * Build: gcc -O3 -ffp-contract=off -fopenmp -fPIC -shared (see __graft_entry__.build_oracle).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXM 12
#define MAXN 3

/* ------------------------------------------------------------------ rows */
static void cars_rows(const float* xs, float u, const float* sig, double gamma_b, float G[][MAXN], float* h) {
    const float kp = 4.0f, kb = 20.0f;
    float p0 = xs[0], p1 = xs[2], p2 = xs[4], p3 = xs[6], p4 = xs[8];
    float v1 = xs[3], v2 = xs[5], v3 = xs[7], v4 = xs[9];
    float a1 = kp * (30.0f - v1), a2 = kp * (30.0f - v2), a4 = kp * (30.0f - v4);
    float d01 = p0 - p1, d12 = p1 - p2, d24 = p2 - p4;
    a1 = a1 - (kb * d01) * (d01 < 6.0f ? 1.0f : 0.0f);
    a2 = a2 - (kb * d12) * (d12 < 6.0f ? 1.0f : 0.0f);
    const float a3 = 0.0f;
    a4 = a4 - (kb * d24) * (d24 < 13.0f ? 1.0f : 0.0f);
    (void)a1;
    float e23 = p2 - p3, e43 = p4 - p3;
    float h13 = 0.5f * ((e23 * e23) - 12.25f), h15 = 0.5f * ((e43 * e43) - 12.25f);
    float h13d = (p3 - p2) * (v3 - v2), h15d = (p3 - p4) * (v3 - v4);
    float c4 = v2 - v3, c5 = p2 - p3, c6 = v3 - v2, c7 = p3 - p2;
    float Lff13 = ((c4 * v2 + c5 * a2) + c6 * v3) + c7 * a3;
    float LfD13 = fabsf(c5) * sig[5] + fabsf(c7) * sig[7];
    float e6 = v3 - v4, e7 = p3 - p4, e8 = v4 - v3, e9 = p4 - p3;
    float Lff15 = ((e6 * v3 + e7 * a3) + e8 * v4) + e9 * a4;
    float LfD15 = fabsf(e7) * sig[7] + fabsf(e9) * sig[9];
    float Lg13 = c7 * 50.0f, Lg15 = e7 * 50.0f;
    float gg = (float)(gamma_b + gamma_b), g2 = (float)(gamma_b * gamma_b);
    h[0] = (((Lff13 - LfD13) + gg * h13d) + g2 * h13) + Lg13 * u;
    h[1] = (((Lff15 - LfD15) + gg * h15d) + g2 * h15) + Lg15 * u;
    G[0][0] = -Lg13; G[0][1] = -200.0f;
    G[1][0] = -Lg15; G[1][1] = -200.0f;
    G[2][0] = 1.0f;  G[2][1] = 0.0f; h[2] = 10.0f - u;
    G[3][0] = -1.0f; G[3][1] = 0.0f; h[3] = -(-10.0f) + u;
}

static void uni_rows(const float* xs, const float* u, const float* mu, const float* sig, double gamma_b,
                     int K, const double* hz, float G[][MAXN], float* h) {
    const float lp = (float)0.03, g = (float)gamma_b;
    float c = (float)cos((double)xs[2]), s = (float)sin((double)xs[2]);
    float px = xs[0] + lp * c, py = xs[1] + lp * s;
    float g00 = c, g01 = -s * lp, g10 = s, g11 = c * lp;
    float mupx = g01 * mu[2] + mu[0], mupy = g11 * mu[2] + mu[1];
    float sgpx = fabsf(g01) * sig[2] + sig[0], sgpy = fabsf(g11) * sig[2] + sig[1];
    const float r2 = (float)((1.2 * 0.6) * (1.2 * 0.6));
    for (int j = 0; j < K; ++j) {
        float dx = px - (float)hz[2 * j], dy = py - (float)hz[2 * j + 1];
        float hs = 0.5f * ((dx * dx + dy * dy) - r2);
        float a0 = dx * g00 + dy * g10, a1 = dx * g01 + dy * g11;
        float t1 = dx * mupx + dy * mupy, t2 = fabsf(dx) * sgpx + fabsf(dy) * sgpy, t3 = a0 * u[0] + a1 * u[1];
        G[j][0] = -a0; G[j][1] = -a1; G[j][2] = -1.0f;
        h[j] = g * ((hs * hs) * hs) + ((t1 - t2) + t3);
    }
    for (int c2 = 0; c2 < 2; ++c2) {
        int r0 = K + 2 * c2;
        for (int k = 0; k < 3; ++k) {
            G[r0][k] = (k == c2) ? 1.0f : 0.0f;
            G[r0 + 1][k] = (k == c2) ? -1.0f : 0.0f;
        }
        h[r0] = 2.5f - u[c2];
        h[r0 + 1] = -(-2.5f) + u[c2];
    }
}

static void normalize(int m, int n, float G[][MAXN], float* h) {
    for (int r = 0; r < m; ++r) {
        float mx = fabsf(G[r][0]);
        for (int k = 1; k < n; ++k) mx = fmaxf(mx, fabsf(G[r][k]));
        float nr = fabsf(h[r]) > mx ? fabsf(h[r]) : mx;
        for (int k = 0; k < n; ++k) G[r][k] = G[r][k] / nr;
        h[r] = h[r] / nr;
    }
}

/* --------------------------------------------- exact QP by enumeration */
/* small dense solve with partial pivoting, A is k x k (k <= 3) */
static int solve_k(int k, double A[MAXN][MAXN], double* b, double* x) {
    for (int c = 0; c < k; ++c) {
        int p = c;
        for (int r = c + 1; r < k; ++r) if (fabs(A[r][c]) > fabs(A[p][c])) p = r;
        if (p != c) {
            for (int j = 0; j < k; ++j) { double t = A[c][j]; A[c][j] = A[p][j]; A[p][j] = t; }
            double t = b[c]; b[c] = b[p]; b[p] = t;
        }
        if (A[c][c] == 0.0) return 0;
        for (int r = c + 1; r < k; ++r) {
            double f = A[r][c] / A[c][c];
            for (int j = c; j < k; ++j) A[r][j] -= f * A[c][j];
            b[r] -= f * b[c];
        }
    }
    for (int i = k - 1; i >= 0; --i) {
        double v = b[i];
        for (int j = i + 1; j < k; ++j) v -= A[i][j] * x[j];
        x[i] = v / A[i][i];
    }
    return 1;
}

/* min 1/2 z' diag(P) z s.t. G z <= h; returns 0 on success.  [nullable]
 * S_out / k_out / lam_out: the active rows (row order) and their multipliers. */
static int qp_exact_as(int m, int n, const double* Pd, float Gf[][MAXN], const float* hf, double* z, int* S_out,
                       int* k_out, double* lam_out);
static int qp_exact(int m, int n, const double* Pd, float Gf[][MAXN], const float* hf, double* z) {
    return qp_exact_as(m, n, Pd, Gf, hf, z, NULL, NULL, NULL);
}
static int qp_exact_as_d(int m, int n, const double* Pd, double G[][MAXN], const double* h, double* z, int* S_out,
                         int* k_out, double* lam_out);
static int qp_exact_as(int m, int n, const double* Pd, float Gf[][MAXN], const float* hf, double* z, int* S_out,
                       int* k_out, double* lam_out) {
    double G[MAXM][MAXN], h[MAXM];
    for (int r = 0; r < m; ++r) {
        h[r] = hf[r];
        for (int k = 0; k < n; ++k) G[r][k] = Gf[r][k];
    }
    return qp_exact_as_d(m, n, Pd, G, h, z, S_out, k_out, lam_out);
}
/* the same on fp64 rows (the Cascade layer's, cbf_qp.py:55-286) */
static int qp_exact_as_d(int m, int n, const double* Pd, double G[][MAXN], const double* h, double* z, int* S_out,
                         int* k_out, double* lam_out) {
    double scale = 1.0, ah = 0.0, ag = 0.0;
    for (int r = 0; r < m; ++r) {
        if (fabs(h[r]) > ah) ah = fabs(h[r]);
        for (int k = 0; k < n; ++k)
            if (fabs(G[r][k]) > ag) ag = fabs(G[r][k]);
    }
    scale += ah + ag;
    const double tol = 1e-10 * scale;
    int S[MAXN];
    for (int k = 0; k <= n; ++k) {
        /* lexicographic combinations of k rows out of m */
        for (int i = 0; i < k; ++i) S[i] = i;
        for (;;) {
            double lam[MAXN] = {0}, zz[MAXN] = {0};
            int ok = 1;
            if (k > 0) {
                double M[MAXN][MAXN], Mc[MAXN][MAXN], rhs[MAXN], rc[MAXN], res[MAXN], corr[MAXN];
                double dprod = 1.0;
                for (int a = 0; a < k; ++a) {
                    for (int b = 0; b < k; ++b) {
                        double acc = 0.0;
                        for (int j = 0; j < n; ++j) acc += G[S[a]][j] / Pd[j] * G[S[b]][j];
                        M[a][b] = acc;
                    }
                    dprod *= M[a][a];
                    rhs[a] = -h[S[a]];
                }
                /* determinant test as the numpy oracle (det > 1e-12 * prod diag) */
                memcpy(Mc, M, sizeof(M));
                double det = 1.0;
                {
                    double T[MAXN][MAXN];
                    memcpy(T, M, sizeof(M));
                    for (int c = 0; c < k; ++c) {
                        int p = c;
                        for (int r = c + 1; r < k; ++r) if (fabs(T[r][c]) > fabs(T[p][c])) p = r;
                        if (p != c) { for (int j = 0; j < k; ++j) { double t = T[c][j]; T[c][j] = T[p][j]; T[p][j] = t; } det = -det; }
                        det *= T[c][c];
                        if (T[c][c] == 0.0) break;
                        for (int r = c + 1; r < k; ++r) {
                            double f = T[r][c] / T[c][c];
                            for (int j = c; j < k; ++j) T[r][j] -= f * T[c][j];
                        }
                    }
                }
                if (!(det > 1e-12 * dprod)) ok = 0;
                if (ok) {
                    memcpy(rc, rhs, sizeof(rhs));
                    ok = solve_k(k, Mc, rc, lam);
                }
                if (ok) { /* one refinement step */
                    for (int a = 0; a < k; ++a) {
                        double acc = rhs[a];
                        for (int b = 0; b < k; ++b) acc -= M[a][b] * lam[b];
                        res[a] = acc;
                    }
                    memcpy(Mc, M, sizeof(M));
                    if (solve_k(k, Mc, res, corr)) for (int a = 0; a < k; ++a) lam[a] += corr[a];
                    for (int j = 0; j < n; ++j) {
                        double acc = 0.0;
                        for (int a = 0; a < k; ++a) acc += G[S[a]][j] * lam[a];
                        zz[j] = -acc / Pd[j];
                    }
                    if (k == n) { /* vertex solve */
                        double A[MAXN][MAXN], b[MAXN];
                        for (int a = 0; a < k; ++a) { for (int j = 0; j < n; ++j) A[a][j] = G[S[a]][j]; b[a] = h[S[a]]; }
                        solve_k(k, A, b, zz);
                    }
                }
            }
            if (ok) {
                double viol = -1e300;
                for (int r = 0; r < m; ++r) {
                    double v = -h[r];
                    for (int j = 0; j < n; ++j) v += G[r][j] * zz[j];
                    if (v > viol) viol = v;
                }
                int dual = 1;
                for (int a = 0; a < k; ++a) if (lam[a] < -tol) dual = 0;
                if (viol <= tol && dual) {
                    for (int j = 0; j < n; ++j) z[j] = zz[j];
                    if (k_out) *k_out = k;
                    for (int a = 0; a < k; ++a) {
                        if (S_out) S_out[a] = S[a];
                        if (lam_out) lam_out[a] = lam[a];
                    }
                    return 0;
                }
            }
            /* next combination */
            int i = k - 1;
            while (i >= 0 && S[i] == m - k + i) --i;
            if (i < 0) break;
            ++S[i];
            for (int j = i + 1; j < k; ++j) S[j] = S[j - 1] + 1;
        }
    }
    for (int j = 0; j < n; ++j) z[j] = NAN;
    return 2;
}

/* ----------------------------------------------------------------- envs */
/* SimulatedCarsEnv.step's physics (envs/simulated_cars_env.py:55-77) for an fp64 action */
static void cars_physics(double* x, double* t, int32_t* step, double a) {
    double vdes0 = 30.0 - 10.0 * sin(0.2 * (*t));
    double acc[5];
    acc[0] = 4.0 * (vdes0 - x[1]);
    for (int i = 1; i < 5; ++i) acc[i] = 4.0 * (30.0 - x[2 * i + 1]);
    double d01 = x[0] - x[2], d12 = x[2] - x[4], d24 = x[4] - x[8];
    acc[1] += (-20.0 * d01) * (d01 < 6.0 ? 1.0 : 0.0);
    acc[2] += (-20.0 * d12) * (d12 < 6.0 ? 1.0 : 0.0);
    acc[4] += (-20.0 * d24) * (d24 < 13.0 ? 1.0 : 0.0);
    for (int i = 0; i < 5; ++i) acc[i] *= 1.1;
    double gu = 50.0 * a, v[5];
    for (int i = 0; i < 5; ++i) v[i] = x[2 * i + 1];
    for (int i = 0; i < 5; ++i) {
        x[2 * i] += 0.02 * (v[i] + 0.0);
        x[2 * i + 1] += 0.02 * (acc[i] + (i == 3 ? gu : 0.0));
    }
    *t = *t + 0.02;
    *step += 1;
}

static void cars_env(double* x, double* t, int32_t* step, float a, float* rew, float* cost, uint8_t* done) {
    double vdes0 = 30.0 - 10.0 * sin(0.2 * (*t));
    double acc[5];
    acc[0] = 4.0 * (vdes0 - x[1]);
    for (int i = 1; i < 5; ++i) acc[i] = 4.0 * (30.0 - x[2 * i + 1]);
    double d01 = x[0] - x[2], d12 = x[2] - x[4], d24 = x[4] - x[8];
    acc[1] += (-20.0 * d01) * (d01 < 6.0 ? 1.0 : 0.0);
    acc[2] += (-20.0 * d12) * (d12 < 6.0 ? 1.0 : 0.0);
    acc[4] += (-20.0 * d24) * (d24 < 13.0 ? 1.0 : 0.0);
    for (int i = 0; i < 5; ++i) acc[i] *= 1.1;
    double gu = 50.0 * (double)a, v[5];
    for (int i = 0; i < 5; ++i) v[i] = x[2 * i + 1];
    for (int i = 0; i < 5; ++i) {
        x[2 * i] += 0.02 * (v[i] + 0.0);
        x[2 * i + 1] += 0.02 * (acc[i] + (i == 3 ? gu : 0.0));
    }
    *t = *t + 0.02;
    *step += 1;
    *done = *step >= 300;
    float a2 = a * a;
    *rew = (-5.0f * fabsf(a2)) / 300.0f;
    double c = 0.0;
    if (x[4] - x[6] < 2.99) c -= 0.1;
    if (x[6] - x[8] < 2.99) c -= 0.1;
    *cost = (float)c;
}

static double goal_dist(const double* x) {
    double d0 = 2.5 - x[0], d1 = 2.5 - x[1];
    return sqrt(d0 * d0 + d1 * d1);
}

static void uni_env(double* x, double* ld, int32_t* step, const float* a, int K, const double* hz, float* rew,
                    float* cost, uint8_t* done) {
    float a0f = a[0] < -1.0f ? -1.0f : (a[0] > 1.0f ? 1.0f : a[0]);
    float a1f = a[1] < -1.0f ? -1.0f : (a[1] > 1.0f ? 1.0f : a[1]);
    double a0 = a0f, a1 = a1f, c = cos(x[2]), s = sin(x[2]);
    x[0] += 0.02 * (0.0 + c * a0);
    x[1] += 0.02 * (0.0 + s * a0);
    x[2] += 0.02 * (0.0 + a1);
    double c2 = cos(x[2]), s2 = sin(x[2]), k = 0.02 * 0.1;
    x[0] -= (k * c2) * c2;
    x[1] -= (k * s2) * c2;
    *step += 1;
    double d = goal_dist(x), r = *ld - d;
    *ld = d;
    int goal = d <= 0.3;
    if (goal) r += 1.0;
    *done = goal || (*step >= 1000);
    *rew = (float)r;
    int hit = 0;
    for (int j = 0; j < K; ++j) {
        double ex = x[0] - hz[2 * j], ey = x[1] - hz[2 * j + 1];
        if (ex * ex + ey * ey < 0.6 * 0.6) hit = 1;
    }
    *cost = hit ? 0.1f : 0.0f;
}

/* ------------------------------------------------------------------ API */
/* CBFQPLayer.get_safe_action with the exact QP, fp32 in / fp32 out. */
int oracle_safe_action(int mode, int K, const double* hz, double gamma_b, int64_t B, const float* x,
                       const float* u, const float* mu, const float* sig, float* out, int nthreads) {
    int fails = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(static) reduction(+ : fails)
    for (int64_t i = 0; i < B; ++i) {
        float G[MAXM][MAXN], h[MAXM];
        double z[MAXN];
        if (mode == 0) {
            cars_rows(x + i * 10, u[i], sig + i * 10, gamma_b, G, h);
            normalize(4, 2, G, h);
            double Pd[2] = {(double)0.1f, (double)10.0f};
            fails += qp_exact(4, 2, Pd, G, h, z) != 0;
            float v = u[i] + (float)z[0];
            out[i] = fminf(fmaxf(v, -10.0f), 10.0f);
        } else {
            uni_rows(x + i * 3, u + i * 2, mu + i * 3, sig + i * 3, gamma_b, K, hz, G, h);
            normalize(K + 4, 3, G, h);
            double Pd[3] = {(double)1.0f, (double)1e-2f, (double)1e5f};
            fails += qp_exact(K + 4, 3, Pd, G, h, z) != 0;
            for (int c = 0; c < 2; ++c) {
                float v = u[2 * i + c] + (float)z[c];
                out[2 * i + c] = fminf(fmaxf(v, -2.5f), 2.5f);
            }
        }
    }
    return fails;
}

/* d(sum w * final)/d u_RL of CBFQPLayer.get_safe_action (oracle.py
 * safe_action_diff_grad restated): the implicit-function derivative of the
 * exact QP on its active set A, through the row normaliser (torch.max routes
 * dN to the first maximal entry of [G_r h_r]) and the clamp mask, fp64:
 *   P dz + dGn' lam + Gn_A' dlam = 0,  Gn_A dz = dhn_A - dGn_A z,
 *   grad_c = sum_a mask_a w_a (delta_ac + dz_a^c). */
static int solve_dense(int k, double A[2 * MAXN][2 * MAXN], double* b, double* x) {
    for (int c = 0; c < k; ++c) {
        int p = c;
        for (int r = c + 1; r < k; ++r) if (fabs(A[r][c]) > fabs(A[p][c])) p = r;
        if (p != c) {
            for (int j = 0; j < k; ++j) { double t = A[c][j]; A[c][j] = A[p][j]; A[p][j] = t; }
            double t = b[c]; b[c] = b[p]; b[p] = t;
        }
        if (A[c][c] == 0.0) return 0;
        for (int r = c + 1; r < k; ++r) {
            double f = A[r][c] / A[c][c];
            for (int j = c; j < k; ++j) A[r][j] -= f * A[c][j];
            b[r] -= f * b[c];
        }
    }
    for (int i = k - 1; i >= 0; --i) {
        double v = b[i];
        for (int j = i + 1; j < k; ++j) v -= A[i][j] * x[j];
        x[i] = v / A[i][i];
    }
    return 1;
}

int oracle_safe_action_grad(int mode, int K, const double* hz, double gamma_b, int64_t B, const float* x,
                            const float* u, const float* mu, const float* sig, const float* w, float* out,
                            double* grad, int nthreads) {
    int fails = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(static) reduction(+ : fails)
    for (int64_t i = 0; i < B; ++i) {
        const int nu = mode == 0 ? 1 : 2, n = nu + 1, m = mode == 0 ? 4 : K + 4;
        const float lo = mode == 0 ? -10.0f : -2.5f, hi = -lo;
        float G[MAXM][MAXN], h[MAXM], Gn[MAXM][MAXN], hn[MAXM];
        double Pd[MAXN];
        if (mode == 0) {
            cars_rows(x + i * 10, u[i], sig + i * 10, gamma_b, G, h);
            Pd[0] = (double)0.1f; Pd[1] = (double)10.0f;
        } else {
            uni_rows(x + i * 3, u + i * 2, mu + i * 3, sig + i * 3, gamma_b, K, hz, G, h);
            Pd[0] = (double)1.0f; Pd[1] = (double)1e-2f; Pd[2] = (double)1e5f;
        }
        memcpy(Gn, G, sizeof(G));
        memcpy(hn, h, sizeof(h));
        normalize(m, n, Gn, hn);
        double z[MAXN], lam[MAXN];
        int S[MAXN], k = 0;
        if (qp_exact_as(m, n, Pd, Gn, hn, z, S, &k, lam) != 0) {
            ++fails;
            for (int c = 0; c < nu; ++c) { out[i * nu + c] = NAN; grad[i * nu + c] = NAN; }
            continue;
        }
        double lamr[MAXM] = {0};
        for (int a = 0; a < k; ++a) lamr[S[a]] = lam[a];
        /* the normaliser's N and which entry torch.max picked (first maximum; |h| wins only if larger) */
        double Nr[MAXM];
        int selh[MAXM];
        for (int r = 0; r < m; ++r) {
            float mx = fabsf(G[r][0]);
            int arg = 0;
            for (int c = 1; c < n; ++c) if (fabsf(G[r][c]) > mx) { mx = fabsf(G[r][c]); arg = c; }
            if (fabsf(h[r]) > mx) { mx = fabsf(h[r]); arg = n; }
            Nr[r] = mx;
            selh[r] = arg == n;
        }
        double J[2][2] = {{0}};
        for (int c = 0; c < nu; ++c) {
            double dhn[MAXM], dGn[MAXM][MAXN];
            for (int r = 0; r < m; ++r) {
                double dh;
                const int k0 = m - 2 * nu;
                if (r < k0) dh = -(double)G[r][c];
                else dh = ((r - k0) / 2 == c) ? (((r - k0) % 2 == 0) ? -1.0 : 1.0) : 0.0;
                const double sgn = h[r] > 0.0f ? 1.0 : (h[r] < 0.0f ? -1.0 : 0.0);
                const double dN = selh[r] ? sgn * dh : 0.0;
                dhn[r] = (dh - (double)hn[r] * dN) / Nr[r];
                for (int j = 0; j < n; ++j) dGn[r][j] = -(double)Gn[r][j] * (dN / Nr[r]);
            }
            double A[2 * MAXN][2 * MAXN] = {{0}}, rhs[2 * MAXN], sol[2 * MAXN];
            for (int j = 0; j < n; ++j) {
                A[j][j] = Pd[j];
                double acc = 0.0;
                for (int r = 0; r < m; ++r) acc += dGn[r][j] * lamr[r];
                rhs[j] = -acc;
            }
            for (int a = 0; a < k; ++a) {
                for (int j = 0; j < n; ++j) {
                    A[j][n + a] = (double)Gn[S[a]][j];
                    A[n + a][j] = (double)Gn[S[a]][j];
                }
                double acc = dhn[S[a]];
                for (int j = 0; j < n; ++j) acc -= dGn[S[a]][j] * z[j];
                rhs[n + a] = acc;
            }
            if (!solve_dense(n + k, A, rhs, sol)) { ++fails; for (int j = 0; j < n; ++j) sol[j] = NAN; }
            for (int a = 0; a < nu; ++a) J[a][c] = (a == c ? 1.0 : 0.0) + sol[a];
        }
        for (int a = 0; a < nu; ++a) {
            const float v = u[i * nu + a] + (float)z[a];
            out[i * nu + a] = fminf(fmaxf(v, lo), hi);
        }
        for (int c = 0; c < nu; ++c) {
            double acc = 0.0;
            for (int a = 0; a < nu; ++a) {
                const float v = u[i * nu + a] + (float)z[a];
                const double mask = (v >= lo && v <= hi) ? 1.0 : 0.0;
                acc += mask * (double)w[i * nu + a] * J[a][c];
            }
            grad[i * nu + c] = acc;
        }
    }
    return fails;
}

/* observations as the policy sees them (fp32): simulated_cars_env.py:143-158,
 * unicycle_env.py:215-231 + obs_compass :260-277 */
static void cars_obs32(const double* xs, float* o) {
    for (int k = 0; k < 10; ++k) o[k] = (float)(xs[k] / ((k & 1) ? 30.0 : 100.0));
}

static void uni_obs32(const double* xs, float* o) {
    double r0 = 2.5 - xs[0], r1 = 2.5 - xs[1];
    double gd = sqrt(r0 * r0 + r1 * r1), c = cos(xs[2]), s = sin(xs[2]);
    double v0 = r0 * c + r1 * s, v1 = r0 * (-s) + r1 * c;
    double nrm = sqrt(v0 * v0 + v1 * v1) + 0.001;
    o[0] = (float)xs[0]; o[1] = (float)xs[1]; o[2] = (float)c; o[3] = (float)s;
    o[4] = (float)(v0 / nrm); o[5] = (float)(v1 / nrm); o[6] = (float)exp(-gd);
}

/* The fused safe step (the hot path bench.py measures): state ->
 * get_state(obs32) -> CBFQPLayer.get_safe_action (mean/sigma NULL -> the
 * DynamicsModel prior, dynamics.py:381-384) -> env.step -> obs; with
 * auto_reset a finished env is reset (simulated_cars_env.py:108-125 /
 * unicycle_env.py:125-143) and its obs is that of the reset state.  The cars
 * reset velocity draw is injected (reset_noise[i] = the N(0, 0.5) sample,
 * NULL -> 0).  obs_out / goal_out may be NULL.  env_action (may be NULL): the
 * action the env steps with instead of the oracle's own safe action (which
 * u_out still reports) -- the parity tests step the oracle env with the
 * device's action, so the env physics is checked exactly on its own. */
int oracle_safe_step_ex(int mode, int K, const double* hz, double gamma_b, int64_t B, double* x, double* aux,
                        int32_t* step, const float* u, const float* mu_in, const float* sig_in, float* u_out,
                        float* rew, float* cost, uint8_t* done, uint8_t* goal_out, float* obs_out, int auto_reset,
                        const double* reset_noise, const float* env_action, int nthreads) {
    int fails = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(static) reduction(+ : fails)
    for (int64_t i = 0; i < B; ++i) {
        float G[MAXM][MAXN], h[MAXM], s32[10], mu[10] = {0}, sig[10];
        double z[MAXN];
        if (mode == 0) {
            double* xs = x + i * 10;
            for (int k = 0; k < 10; ++k) {
                double sc = (k & 1) ? 30.0 : 100.0;
                float o = (float)(xs[k] / sc);
                s32[k] = (float)((double)o * sc);
                sig[k] = sig_in ? sig_in[i * 10 + k] : ((k & 1) ? (float)0.2 : 0.0f);
            }
            cars_rows(s32, u[i], sig, gamma_b, G, h);
            normalize(4, 2, G, h);
            double Pd[2] = {(double)0.1f, (double)10.0f};
            fails += qp_exact(4, 2, Pd, G, h, z) != 0;
            float v = u[i] + (float)z[0];
            float a = fminf(fmaxf(v, -10.0f), 10.0f);
            u_out[i] = a;
            if (env_action) a = env_action[i];
            cars_env(xs, aux + i, step + i, a, rew + i, cost + i, done + i);
            if (goal_out) goal_out[i] = 0;
            if (auto_reset && done[i]) {
                const double nz = reset_noise ? reset_noise[i] : 0.0;
                const double p0[5] = {34.0, 28.0, 22.0, 16.0, 10.0};
                for (int c = 0; c < 5; ++c) { xs[2 * c] = p0[c]; xs[2 * c + 1] = 30.0 + nz; }
                xs[7] = 35.0;
                aux[i] = 0.0;
                step[i] = 0;
            }
            if (obs_out) cars_obs32(xs, obs_out + i * 10);
        } else {
            double* xs = x + i * 3;
            float o2 = (float)cos(xs[2]), o3 = (float)sin(xs[2]);
            s32[0] = (float)xs[0];
            s32[1] = (float)xs[1];
            s32[2] = (float)atan2((double)o3, (double)o2);
            for (int k = 0; k < 3; ++k) {
                mu[k] = mu_in ? mu_in[i * 3 + k] : 0.0f;
                sig[k] = sig_in ? sig_in[i * 3 + k] : (float)0.2;
            }
            uni_rows(s32, u + 2 * i, mu, sig, gamma_b, K, hz, G, h);
            normalize(K + 4, 3, G, h);
            double Pd[3] = {(double)1.0f, (double)1e-2f, (double)1e5f};
            fails += qp_exact(K + 4, 3, Pd, G, h, z) != 0;
            float a[2];
            for (int c = 0; c < 2; ++c) {
                float v = u[2 * i + c] + (float)z[c];
                a[c] = fminf(fmaxf(v, -2.5f), 2.5f);
                u_out[2 * i + c] = a[c];
                if (env_action) a[c] = env_action[2 * i + c];
            }
            uni_env(xs, aux + i, step + i, a, K, hz, rew + i, cost + i, done + i);
            if (goal_out) goal_out[i] = goal_dist(xs) <= 0.3;
            if (auto_reset && done[i]) {
                xs[0] = -2.5; xs[1] = -2.5; xs[2] = 0.0;
                aux[i] = goal_dist(xs);
                step[i] = 0;
            }
            if (obs_out) uni_obs32(xs, obs_out + i * 7);
        }
    }
    return fails;
}

/* The fused step with the prior, no auto-reset (bench.py's cpu_baseline). */
int oracle_safe_step(int mode, int K, const double* hz, double gamma_b, int64_t B, double* x, double* aux,
                     int32_t* step, const float* u, float* u_out, float* rew, float* cost, uint8_t* done,
                     int nthreads) {
    return oracle_safe_step_ex(mode, K, hz, gamma_b, B, x, aux, step, u, NULL, NULL, u_out, rew, cost, done, NULL,
                               NULL, 0, NULL, NULL, nthreads);
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------ config 1: the Cascade closed loop */
/* BASELINE.json config 1, the reference's own demo (envs/simulated_cars_env.py:161-228): one SimulatedCars
 * env from reset (positions 34, 28, 22, 16, 10; velocities 30 + noise, car 3 at 35; :108-125) for `steps`
 * steps of
 *   obs = x / [100, 30] (:143-158) -> state = obs * [100, 30] (DynamicsModel.get_state, dynamics.py:190-232,
 *   fp64) -> the hand controller (:195-199) -> CascadeCBFLayer.get_u_safe (cbf_qp.py:29-53: the cars rows
 *   of :149-219 + :224-238 with no robust term and gamma_b, P = diag(0.1, 10), q = 0; rows normalised by
 *   max(|G_r|, |h_r|) as :270-273; the exact QP that quadprog returns at :276) -> env.step(u_nom + u_safe).
 * u_nom_out, u_safe_out (steps,), x_out ((steps + 1) x 10): [nullable].  Returns 0, or 1 + the step whose
 * QP had no solution. */
int oracle_cars_cascade_loop(double noise, int steps, double gamma_b, double* u_nom_out, double* u_safe_out,
                             double* x_out) {
    double x[10] = {34.0, 30.0 + noise, 28.0, 30.0 + noise, 22.0, 30.0 + noise, 16.0, 35.0, 10.0, 30.0 + noise};
    double t = 0.0;
    int32_t st = 0;
    if (x_out) memcpy(x_out, x, sizeof x);
    for (int k = 0; k < steps; ++k) {
        double s[10];
        for (int i = 0; i < 10; ++i) {
            const double o = (i & 1) ? x[i] / 30.0 : x[i] / 100.0;
            s[i] = (i & 1) ? o * 30.0 : o * 100.0;
        }
        double u = (s[4] - s[6] - 0.4) * ((s[4] - s[6] - 0.4) < 0 ? 1.0 : 0.0);
        u += (s[8] - s[6] + 0.4) * ((s[8] - s[6] + 0.4) > 0 ? 1.0 : 0.0);
        /* Cascade rows (fp64) */
        double p[5], v[5], a[5];
        for (int i = 0; i < 5; ++i) { p[i] = s[2 * i]; v[i] = s[2 * i + 1]; a[i] = 4.0 * (30.0 - v[i]); }
        const double d01 = p[0] - p[1], d12 = p[1] - p[2], d24 = p[2] - p[4];
        a[1] = a[1] - 20.0 * d01 * (d01 < 6.0 ? 1.0 : 0.0);
        a[2] = a[2] - 20.0 * d12 * (d12 < 6.0 ? 1.0 : 0.0);
        a[3] = 0.0;
        a[4] = a[4] - 20.0 * d24 * (d24 < 13.0 ? 1.0 : 0.0);
        const double h13 = 0.5 * ((p[2] - p[3]) * (p[2] - p[3]) - 3.5 * 3.5);
        const double h15 = 0.5 * ((p[4] - p[3]) * (p[4] - p[3]) - 3.5 * 3.5);
        const double h13d = (p[3] - p[2]) * (v[3] - v[2]), h15d = (p[3] - p[4]) * (v[3] - v[4]);
        const double Lff13 = (v[2] - v[3]) * v[2] + (p[2] - p[3]) * a[2] + (v[3] - v[2]) * v[3] + (p[3] - p[2]) * a[3];
        const double Lff15 = (v[3] - v[4]) * v[3] + (p[3] - p[4]) * a[3] + (v[4] - v[3]) * v[4] + (p[4] - p[3]) * a[4];
        const double Lg13 = 50.0 * (p[3] - p[2]), Lg15 = 50.0 * (p[3] - p[4]);
        double G[MAXM][MAXN] = {{0}}, h[MAXM];
        h[0] = Lff13 + (gamma_b + gamma_b) * h13d + gamma_b * gamma_b * h13 + Lg13 * u;
        h[1] = Lff15 + (gamma_b + gamma_b) * h15d + gamma_b * gamma_b * h15 + Lg15 * u;
        G[0][0] = -Lg13; G[1][0] = -Lg15; G[0][1] = G[1][1] = -2e2;
        G[2][0] = 1.0; h[2] = 10.0 - u;
        G[3][0] = -1.0; h[3] = 10.0 + u;
        for (int r = 0; r < 4; ++r) { /* cbf_qp.py:270-273 */
            double nr = fabs(h[r]);
            for (int c = 0; c < 2; ++c) if (fabs(G[r][c]) > nr) nr = fabs(G[r][c]);
            for (int c = 0; c < 2; ++c) G[r][c] = G[r][c] / nr;
            h[r] = h[r] / nr;
        }
        const double Pd[2] = {0.1, 1e1};
        double z[MAXN];
        if (qp_exact_as_d(4, 2, Pd, G, h, z, NULL, NULL, NULL)) return k + 1;
        if (u_nom_out) u_nom_out[k] = u;
        if (u_safe_out) u_safe_out[k] = z[0];
        cars_physics(x, &t, &st, u + z[0]);
        if (x_out) memcpy(x_out + 10 * (k + 1), x, sizeof x);
    }
    return 0;
}
