// rcbf_qp.hip -- generic QP forward (fp32) + C-ABI: rcbf_qp_solve and
// rcbf_qp_solve_saved (CBFQPLayer.solve_qp / cbf_layer, diff_cbf_qp.py:81-144).
// The machinery is in rcbf_qp_common.hpp; rcbf_qp_f64.hip holds the fp64
// forward, rcbf_qp_bwd.hip the backward, rcbf_cascade.hip the Cascade layer.
#include "rcbf_qp_common.hpp"

using namespace rcbf;
using namespace rcbf_qp;

extern "C" {

int rcbf_qp_solve(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P, const float* q,
                  const float* G, const float* h, int32_t normalize, float* z_out, double* lam_out,
                  int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    return qp_solve_launch<float>(prm, B, n, m, P, q, G, h, normalize, z_out, lam_out, status_out, fail_flag, stream);
}


int rcbf_qp_solve_saved(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const float* P, const float* q,
                        const float* G, const float* h, int32_t normalize, float* z_out, double* z64_saved,
                        int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    if (!z64_saved) return RCBF_E_NULL;
    return qp_solve_launch<float>(prm, B, n, m, P, q, G, h, normalize, z_out, nullptr, status_out, fail_flag, stream,
                                  z64_saved);
}

}  // extern "C"
