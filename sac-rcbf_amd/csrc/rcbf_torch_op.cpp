// rcbf_torch_op.cpp -- the SAC-update safe action as a C++ autograd op.
//
// RCBF_SAC.get_safe_action (rcbf_sac/sac_cbf.py:218-238) runs on every SGD
// update with gradients flowing into the policy (sac_cbf.py:147-158).  The
// Python torch.autograd.Function around the two launches (rcbf_amd
// diff_cbf_qp._SafeAction) costs tens of microseconds of host time per
// call; this op is the same forward / backward pair as a
// torch::autograd::Function, so the only host work left is the two C-ABI
// launches and the reference's NaN check (diff_cbf_qp.py:141-143: one 4-byte
// read of the device fail flag, then Exception('QP Failed to solve')).
//
// When the action needs a gradient the forward is the Jacobian-keeping
// launch (rcbf_[obs_]safe_action_jac: the same u_out, plus d final / d u_rl
// per row, as qpth's QPFunction keeps its solution), and the backward is one
// elementwise launch (rcbf_safe_action_apply_jac) instead of a second solve;
// a forward under no_grad (acting) is the plain launch.
//
// Like csrc/rcbf_pyfast.cpp it links nothing of ours: bind() receives the
// addresses of the entry points from the library ctypes loaded
// (rcbf_amd._lib).  Host C++ only.
#include <torch/extension.h>

#include <c10/hip/HIPStream.h>

#include <cstring>

#include "rcbf_hip.h"

namespace {

using FwdFn = decltype(&rcbf_safe_action);
using BwdFn = decltype(&rcbf_safe_action_backward);
using JacFn = decltype(&rcbf_safe_action_jac);
using ApplyFn = decltype(&rcbf_safe_action_apply_jac);

FwdFn g_fwd[2] = {nullptr, nullptr};  // [0] state input (rcbf_safe_action), [1] obs input (rcbf_obs_safe_action)
BwdFn g_bwd[2] = {nullptr, nullptr};
JacFn g_jac[2] = {nullptr, nullptr};
ApplyFn g_apply = nullptr;

hipStream_t current_stream(const torch::Tensor& t) {
    return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

// mean / sigma: a zero-element tensor stands for NULL (the in-kernel prior)
const float* fptr(const torch::Tensor& t) { return t.numel() ? t.data_ptr<float>() : nullptr; }

void check_rc(int rc, const char* what) {
    TORCH_CHECK(rc == 0, what, " failed: ", rc == RCBF_E_BAD_MODE ? "RCBF_E_BAD_MODE"
                                            : rc == RCBF_E_BAD_SHAPE ? "RCBF_E_BAD_SHAPE"
                                            : rc == RCBF_E_NULL      ? "RCBF_E_NULL"
                                                                     : "hipError_t ", rc);
}

struct SafeActionOp : public torch::autograd::Function<SafeActionOp> {
    // x: (B, n_o) observations (from_obs) or (B, n_s) states; u: (B, n_u) f32; mu/sigma: empty -> prior
    // want_jac: the caller's u requires grad with grad mode on -> keep the Jacobian for the backward
    static torch::Tensor forward(torch::autograd::AutogradContext* ctx, torch::Tensor x, torch::Tensor u,
                                 torch::Tensor mu, torch::Tensor sigma, int64_t prm, int64_t flag_addr,
                                 bool from_obs, bool want_jac) {
        const int k = from_obs ? 1 : 0;
        TORCH_CHECK(g_fwd[k] && g_bwd[k] && g_jac[k] && g_apply, "_rcbf_torch: bind() the library entry points first");
        auto out = torch::empty_like(u);
        auto* flag = reinterpret_cast<int32_t*>(flag_addr);
        const auto* p = reinterpret_cast<const rcbf_params*>(prm);
        torch::Tensor jac;
        if (want_jac) {
            jac = torch::empty({u.size(0), u.size(1), u.size(1)}, u.options().dtype(torch::kFloat64));
            check_rc(g_jac[k](p, x.size(0), x.data_ptr<float>(), u.data_ptr<float>(), fptr(mu), fptr(sigma),
                              out.data_ptr<float>(), jac.data_ptr<double>(), nullptr, flag, current_stream(x)),
                     from_obs ? "rcbf_obs_safe_action_jac" : "rcbf_safe_action_jac");
        } else {
            check_rc(g_fwd[k](p, x.size(0), x.data_ptr<float>(), u.data_ptr<float>(), fptr(mu), fptr(sigma),
                              out.data_ptr<float>(), nullptr, flag, current_stream(x)),
                     from_obs ? "rcbf_obs_safe_action" : "rcbf_safe_action");
        }
        if (flag) {
            // the reference's NaN check (one device -> host read; it syncs there too)
            auto f = torch::from_blob(flag, {1}, torch::TensorOptions().dtype(torch::kInt32).device(x.device()));
            if (f.item<int32_t>() != 0) {
                f.zero_();
                throw std::runtime_error("QP Failed to solve");
            }
        }
        if (want_jac) {
            ctx->save_for_backward({jac});
            ctx->saved_data["jac"] = true;
            return out;
        }
        ctx->save_for_backward({x, u, mu, sigma});
        // the backward must not depend on the caller's layer object staying
        // alive: keep a private copy of the parameter block with the graph
        auto pcopy = torch::empty({(int64_t)sizeof(rcbf_params)}, torch::TensorOptions().dtype(torch::kUInt8));
        std::memcpy(pcopy.data_ptr(), reinterpret_cast<const void*>(prm), sizeof(rcbf_params));
        ctx->saved_data["prm"] = pcopy;
        ctx->saved_data["from_obs"] = from_obs;
        ctx->saved_data["jac"] = false;
        return out;
    }

    static torch::autograd::tensor_list backward(torch::autograd::AutogradContext* ctx,
                                                 torch::autograd::tensor_list grads) {
        auto saved = ctx->get_saved_variables();
        if (ctx->saved_data["jac"].toBool()) {  // the forward kept d final / d u_rl
            auto jac = saved[0];
            auto g = grads[0].to(torch::kFloat32).contiguous();
            auto gu = torch::empty_like(g);
            check_rc(g_apply(jac.size(0), (int32_t)jac.size(1), jac.data_ptr<double>(), g.data_ptr<float>(),
                             gu.data_ptr<float>(), current_stream(jac)),
                     "rcbf_safe_action_apply_jac");
            return {torch::Tensor(), gu, torch::Tensor(), torch::Tensor(), torch::Tensor(), torch::Tensor(),
                    torch::Tensor(), torch::Tensor()};
        }
        auto x = saved[0], u = saved[1], mu = saved[2], sigma = saved[3];
        const bool from_obs = ctx->saved_data["from_obs"].toBool();
        const auto pcopy = ctx->saved_data["prm"].toTensor();
        const auto* prm = reinterpret_cast<const rcbf_params*>(pcopy.data_ptr());
        auto g = grads[0].to(torch::kFloat32).contiguous();
        auto gu = torch::empty_like(u);
        check_rc(g_bwd[from_obs ? 1 : 0](prm, x.size(0), x.data_ptr<float>(),
                                         u.data_ptr<float>(), fptr(mu), fptr(sigma), g.data_ptr<float>(),
                                         gu.data_ptr<float>(), current_stream(x)),
                 from_obs ? "rcbf_obs_safe_action_backward" : "rcbf_safe_action_backward");
        return {torch::Tensor(), gu, torch::Tensor(), torch::Tensor(), torch::Tensor(), torch::Tensor(),
                torch::Tensor(), torch::Tensor()};
    }
};

void bind(int64_t safe_action, int64_t safe_action_bwd, int64_t obs_safe_action, int64_t obs_safe_action_bwd,
          int64_t safe_action_jac, int64_t obs_safe_action_jac, int64_t apply_jac) {
    g_fwd[0] = reinterpret_cast<FwdFn>(safe_action);
    g_bwd[0] = reinterpret_cast<BwdFn>(safe_action_bwd);
    g_fwd[1] = reinterpret_cast<FwdFn>(obs_safe_action);
    g_bwd[1] = reinterpret_cast<BwdFn>(obs_safe_action_bwd);
    g_jac[0] = reinterpret_cast<JacFn>(safe_action_jac);
    g_jac[1] = reinterpret_cast<JacFn>(obs_safe_action_jac);
    g_apply = reinterpret_cast<ApplyFn>(apply_jac);
}

// safe_action(x, u, mu, sigma, prm_addr, flag_addr, from_obs): inputs already f32, contiguous, on one device
torch::Tensor safe_action(torch::Tensor x, torch::Tensor u, c10::optional<torch::Tensor> mu,
                          c10::optional<torch::Tensor> sigma, int64_t prm, int64_t flag_addr, bool from_obs) {
    TORCH_CHECK(x.is_cuda() && u.is_cuda() && x.scalar_type() == torch::kFloat32 &&
                    u.scalar_type() == torch::kFloat32 && x.is_contiguous() && u.is_contiguous() &&
                    x.device() == u.device() && x.dim() == 2 && u.dim() == 2 && x.size(0) == u.size(0),
                "_rcbf_torch.safe_action: x (B, n) and u (B, n_u) must be contiguous f32 tensors on one HIP device");
    auto none = torch::empty({0}, x.options());
    const bool want_jac = u.requires_grad() && torch::GradMode::is_enabled();
    return SafeActionOp::apply(x, u, mu.has_value() ? *mu : none, sigma.has_value() ? *sigma : none, prm, flag_addr,
                               from_obs, want_jac);
}

}  // namespace

PYBIND11_MODULE(_rcbf_torch, m) {
    m.doc() = "SAC-update safe action (rcbf_[obs_]safe_action + backward) as a C++ autograd op";
    m.def("bind", &bind, "bind the entry points of the loaded librcbf_hip.so");
    m.def("safe_action", &safe_action, "differentiable safe action w.r.t. u");
}
