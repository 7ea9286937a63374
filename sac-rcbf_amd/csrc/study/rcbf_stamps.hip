// rcbf_stamps.hip -- STUDY BUILD ONLY (not part of librcbf_hip.so): the fused
// safe step instantiated with phase timestamps (Stamps<true>, s_memtime per
// wave at phase boundaries), for scripts/stamps.py.  Built on demand into
// build/study/librcbf_stamps.so; the product kernel is the same template with
// the stamps compiled out.  RCBF_STUDY_QP_STAMPS adds the unicycle QP's
// per-stage record (rcbf_device.hpp) into a second buffer.
#define RCBF_STUDY_QP_STAMPS 1
#include <hip/hip_runtime.h>
__device__ unsigned long long* rcbf_qp_stamp_buf = nullptr;
#include "../rcbf_safe_step.hpp"

using namespace rcbf;

extern "C" int rcbf_study_safe_step_stamps(const rcbf_params* prm, int64_t B, double* x, double* aux, int32_t* step,
                                           uint32_t* episode, const float* u_rl, float* obs_out, float* u_out,
                                           float* reward, float* cost, uint8_t* done, unsigned long long* stamps,
                                           int32_t auto_reset, uint64_t seed, hipStream_t stream) {
    if (int e = check_prm(prm)) return e;
    if (B <= 0 || !stamps) return RCBF_E_BAD_SHAPE;
    RCBF_DISPATCH(prm, hipLaunchKernelGGL((k_safe_step<SOLVER_, MODE_, K_, true>), dim3(grid_for_envs(B)), dim3(kBlock),
                                          0, stream, B, x, aux, step, u_rl, episode, nullptr, nullptr, obs_out, u_out,
                                          reward, cost, done, nullptr, nullptr, nullptr, auto_reset, seed, (int64_t)0,
                                          *prm, 0, stamps));
    return launch_status();
}

// the QP record's buffer (16 words per wave; null: off)
extern "C" int rcbf_study_set_qp_stamps(unsigned long long* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(rcbf_qp_stamp_buf), &buf, sizeof(buf));
}
