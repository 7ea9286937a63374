// rcbf_cascade.hip -- the Cascade layer (CascadeCBFLayer.get_u_safe,
// cbf_qp.py:29-53) + C-ABI: rcbf_cascade_u_safe.
#include "rcbf_common.hpp"

using namespace rcbf;

namespace {

template <int SOLVER, int MODE, int K>
__device__ __forceinline__ void cascade_one(const rcbf_params& prm, int64_t i, const double* __restrict__ un,
                                            const double* __restrict__ x, const double* __restrict__ mu,
                                            const double* __restrict__ sigma, double* __restrict__ u_out,
                                            int32_t* __restrict__ status_out, int32_t* fail_flag,
                                            double* __restrict__ eps_out) {
    using D = Dims<MODE, K>;
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
    if (eps_out) eps_out[i] = res.z[D::NU];  // the slack, sol[0][-1] (cbf_qp.py:278, 283-284)
    report(res.status, status_out, i, fail_flag);
}

template <int SOLVER, int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_cascade(rcbf_params prm, int64_t B, const double* __restrict__ un,
                                                    const double* __restrict__ x, const double* __restrict__ mu,
                                                    const double* __restrict__ sigma, double* __restrict__ u_out,
                                                    int32_t* __restrict__ status_out, int32_t* fail_flag,
                                                    double* __restrict__ eps_out) {
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= B) return;
    cascade_one<SOLVER, MODE, K>(prm, i, un, x, mu, sigma, u_out, status_out, fail_flag, eps_out);
}

// B <= kBlock in ONE workgroup, then a completion word in pinned host memory (rcbf_cascade_u_safe_sync):
// the single-sample get_u_safe of the reference's loop (envs/simulated_cars_env.py:213) without a copy or a
// stream synchronisation; the inputs and outputs may live in pinned host memory (read and written in place)
template <int SOLVER, int MODE, int K>
__global__ void __launch_bounds__(kBlock) k_cascade_sync(rcbf_params prm, int64_t B, const double* __restrict__ un,
                                                         const double* __restrict__ x, const double* __restrict__ mu,
                                                         const double* __restrict__ sigma,
                                                         double* __restrict__ u_out, int32_t* __restrict__ status_out,
                                                         double* __restrict__ eps_out, uint32_t* done_word,
                                                         uint32_t seq) {
    const int64_t i = threadIdx.x;
    if (i < B) cascade_one<SOLVER, MODE, K>(prm, i, un, x, mu, sigma, u_out, status_out, nullptr, eps_out);
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();  // every lane's outputs land before the word
        __hip_atomic_store(done_word, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

extern "C" {

int rcbf_cascade_u_safe(const rcbf_params* prm, int64_t B, const double* u_nom, const double* x, const double* mu,
                        const double* sigma, double* u_safe_out, int32_t* status_out, int32_t* fail_flag,
                        double* eps_out, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 0) return RCBF_E_BAD_SHAPE;
    if (B == 0) return 0;
    if (!x || !u_nom || !u_safe_out) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_cascade<SOLVER_, MODE_, K_>), dim3(grid_for(B)), dim3(kBlock), 0, stream,
                                          *prm, B, u_nom, x, mu, sigma, u_safe_out, status_out, fail_flag, eps_out));
    return launch_status();
}

int rcbf_cascade_u_safe_sync(const rcbf_params* prm, int64_t B, const double* u_nom, const double* x,
                             const double* mu, const double* sigma, double* u_safe_out, int32_t* status_out,
                             double* eps_out, uint32_t* done_word, uint32_t seq, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B < 1 || B > kBlock) return RCBF_E_BAD_SHAPE;
    if (!x || !u_nom || !u_safe_out || !done_word) return RCBF_E_NULL;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_cascade_sync<SOLVER_, MODE_, K_>), dim3(1), dim3(kBlock), 0, stream,
                                          *prm, B, u_nom, x, mu, sigma, u_safe_out, status_out, eps_out, done_word,
                                          seq));
    if (int rc = launch_status()) return rc;
    // poll the word; every 4096 polls ask the stream, so a failed kernel returns its error instead of spinning
    volatile uint32_t* w = done_word;
    for (uint32_t n = 1;; ++n) {
        if (*w == seq) return 0;
        __builtin_ia32_pause();
        if ((n & 4095) == 0) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) return *w == seq ? 0 : (int)hipErrorUnknown;
            if (q != hipErrorNotReady) return (int)q;
        }
    }
}

}  // extern "C"
