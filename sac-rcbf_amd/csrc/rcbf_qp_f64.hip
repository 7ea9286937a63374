// rcbf_qp_f64.hip -- generic QP forward in fp64 + C-ABI: rcbf_qp_solve_f64
// (CascadeCBFLayer.solve_qp, cbf_qp.py:242-286).  Machinery in rcbf_qp_common.hpp.
#include "rcbf_qp_common.hpp"

using namespace rcbf;
using namespace rcbf_qp;

extern "C" {

int rcbf_qp_solve_f64(const rcbf_params* prm, int64_t B, int32_t n, int32_t m, const double* P, const double* q,
                      const double* G, const double* h, int32_t normalize, double* z_out, double* lam_out,
                      int32_t* status_out, int32_t* fail_flag, hipStream_t stream) {
    return qp_solve_launch<double>(prm, B, n, m, P, q, G, h, normalize, z_out, lam_out, status_out, fail_flag,
                                   stream);
}

}  // extern "C"
