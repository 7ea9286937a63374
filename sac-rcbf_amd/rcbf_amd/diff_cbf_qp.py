"""Drop-in `CBFQPLayer` (rcbf_sac/diff_cbf_qp.py:10-395) on the HIP kernels.

Same constructor, attributes, methods and exceptions as the reference; the
whole get_safe_action (build -> row normalise -> fp64 QP -> clamp) is ONE
kernel launch (rcbf_safe_action) and its backward w.r.t. the action is one
more (rcbf_safe_action_backward).  No qpth, no CPU path: inputs on the CPU are
moved to the HIP device for the launch and the result is moved back.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .dynamics import DYNAMICS_MODE
from .params import make_params

_QP_FAILED = "QP Failed to solve"


def _dev():
    if not torch.cuda.is_available():
        raise RuntimeError("CBFQPLayer needs a HIP device (MI355X); there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def _f32(t, dev):
    if not torch.is_tensor(t):
        t = torch.as_tensor(np.asarray(t))
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


def _f32_keep_grad(t, dev):
    """_f32 for inputs that may carry autograd history (kept differentiable)."""
    if torch.is_tensor(t) and t.requires_grad:
        t = t.to(device=dev, dtype=torch.float32)
        return t if t.is_contiguous() else t.contiguous()
    return _f32(t, dev)


def _fail_flag(layer, device):
    """The layer's persistent device fail-flag word for `device` (zero between
    calls: a call that sees it set clears it before raising), so a call costs
    no fill launch."""
    flags = layer.__dict__.setdefault("_fail_flags", {})
    f = flags.get(device)
    if f is None:
        f = flags[device] = torch.zeros(1, dtype=torch.int32, device=device)
    return f


def _raise_if_failed(flag):
    bits = int(flag.item())  # one 4-byte read (the reference syncs here too, :141)
    if bits:
        flag.zero_()
        raise Exception(_QP_FAILED)


class _SafeAction(torch.autograd.Function):
    """final = clamp(u + QP(u)[:n_u]);  grad flows to `u` only, like the
    reference whose state/mean/sigma arrive detached (dynamics.py:211,362).
    When u needs a gradient the forward keeps d final / d u per row
    (rcbf_[obs_]safe_action_jac) and the backward is rcbf_safe_action_apply_jac."""

    @staticmethod
    def forward(ctx, layer, x, u, mu, sigma, from_obs=False):
        lib = _lib.load()
        B = x.shape[0]
        out = torch.empty_like(u)
        flag = _fail_flag(layer, x.device) if layer.check_failures else None
        want_jac = bool(ctx.needs_input_grad[2])
        if want_jac:
            jac = torch.empty(B, u.shape[1], u.shape[1], dtype=torch.float64, device=u.device)
            fn = lib.rcbf_obs_safe_action_jac if from_obs else lib.rcbf_safe_action_jac
            rc = fn(ctypes.byref(layer._prm), B, _lib.ptr(x), _lib.ptr(u), _lib.ptr(mu), _lib.ptr(sigma),
                    _lib.ptr(out), _lib.ptr(jac), None, _lib.ptr(flag), _lib.stream_of(x.device))
            _lib.check(rc, "rcbf_obs_safe_action_jac" if from_obs else "rcbf_safe_action_jac")
        else:
            fn = lib.rcbf_obs_safe_action if from_obs else lib.rcbf_safe_action
            rc = fn(ctypes.byref(layer._prm), B, _lib.ptr(x), _lib.ptr(u), _lib.ptr(mu), _lib.ptr(sigma),
                    _lib.ptr(out), None, _lib.ptr(flag), _lib.stream_of(x.device))
            _lib.check(rc, "rcbf_obs_safe_action" if from_obs else "rcbf_safe_action")
        if layer.check_failures:
            _raise_if_failed(flag)
        ctx.layer = layer
        ctx.from_obs = from_obs
        ctx.want_jac = want_jac
        if want_jac:
            ctx.save_for_backward(jac)
        else:
            ctx.save_for_backward(x, u, mu, sigma)
        return out

    @staticmethod
    def backward(ctx, grad):
        lib = _lib.load()
        g = grad.contiguous().to(torch.float32)
        if ctx.want_jac:
            (jac,) = ctx.saved_tensors
            gu = torch.empty_like(g)
            rc = lib.rcbf_safe_action_apply_jac(jac.shape[0], jac.shape[1], _lib.ptr(jac), _lib.ptr(g), _lib.ptr(gu),
                                                _lib.stream_of(jac.device))
            _lib.check(rc, "rcbf_safe_action_apply_jac")
            return None, None, gu, None, None, None
        x, u, mu, sigma = ctx.saved_tensors
        gu = torch.empty_like(u)
        fn = lib.rcbf_obs_safe_action_backward if ctx.from_obs else lib.rcbf_safe_action_backward
        rc = fn(ctypes.byref(ctx.layer._prm), x.shape[0], _lib.ptr(x), _lib.ptr(u), _lib.ptr(mu), _lib.ptr(sigma),
                _lib.ptr(g), _lib.ptr(gu), _lib.stream_of(x.device))
        _lib.check(rc, "rcbf_obs_safe_action_backward" if ctx.from_obs else "rcbf_safe_action_backward")
        return None, None, gu, None, None, None


def safe_action_op(layer, x, u, mu, sigma, from_obs=False):
    """final = clamp(u + QP(u)[:n_u]) with autograd w.r.t. u: the C++ autograd
    op (csrc/rcbf_torch_op.cpp) when it is built, else the Python Function;
    both launch the same two C-ABI entry points and raise the reference's
    Exception('QP Failed to solve') after one flag read."""
    op = _lib.torch_op()
    if op is None:
        return _SafeAction.apply(layer, x, u, mu, sigma, from_obs)
    flag = _fail_flag(layer, x.device) if layer.check_failures else None
    return op.safe_action(x, u, mu, sigma, ctypes.addressof(layer._prm), 0 if flag is None else flag.data_ptr(),
                          bool(from_obs))


class _QP(torch.autograd.Function):
    """z = QP(P, q, G, h) (optionally on row-normalised [G h]); backward is
    rcbf_qp_backward: the implicit-KKT adjoint on the exact active set (what
    qpth's QPFunction.backward approximates) w.r.t. P, q, G, h, pulled back
    through the normaliser like torch autograd through diff_cbf_qp.py:103-106."""

    @staticmethod
    def forward(ctx, layer, prm, normalize, P, q, G, h):
        lib = _lib.load()
        B, m, n = G.shape
        z = torch.empty(B, n, device=G.device)
        z64 = torch.empty(B, n, dtype=torch.float64, device=G.device)  # kept for the backward, like qpth's zhats
        flag = _fail_flag(layer, G.device)
        rc = lib.rcbf_qp_solve_saved(ctypes.byref(prm), B, n, m, _lib.ptr(P), _lib.ptr(q), _lib.ptr(G),
                                     _lib.ptr(h), int(normalize), _lib.ptr(z), _lib.ptr(z64), None, _lib.ptr(flag),
                                     _lib.stream_of(G.device))
        _lib.check(rc, "rcbf_qp_solve_saved")
        _raise_if_failed(flag)
        ctx.prm = prm
        ctx.normalize = normalize
        ctx.save_for_backward(P, q, G, h, z64)
        return z

    @staticmethod
    def backward(ctx, grad_z):
        P, q, G, h, z64 = ctx.saved_tensors
        B, m, n = G.shape
        need = ctx.needs_input_grad
        gz = grad_z.to(torch.float32).contiguous()
        # inputs: layer, prm, normalize, P, q, G, h
        gP = torch.empty_like(P) if need[3] else None
        gq = torch.empty(B, n, device=G.device) if (need[4] and q is not None) else None
        gG = torch.empty_like(G) if need[5] else None
        gh = torch.empty_like(h) if need[6] else None
        rc = _lib.load().rcbf_qp_backward_saved(ctypes.byref(ctx.prm), B, n, m, _lib.ptr(P), _lib.ptr(q),
                                                _lib.ptr(G), _lib.ptr(h), int(ctx.normalize), _lib.ptr(z64),
                                                _lib.ptr(gz), _lib.ptr(gP), _lib.ptr(gq), _lib.ptr(gG), _lib.ptr(gh),
                                                _lib.stream_of(G.device))
        _lib.check(rc, "rcbf_qp_backward_saved")
        return None, None, None, gP, gq, gG, gh


def _divide_rows_in_place(Gs, hs):
    """The caller-visible side effect of the reference's solve_qp
    (diff_cbf_qp.py:103-105): Gs divided in place by max |[G h]| of its row,
    with torch's own division, so the caller sees the very rows qpth saw.
    With autograd recording, the reference's own ops: the division and its
    norm are differentiated (a leaf that requires grad raises torch's
    in-place RuntimeError, as the reference does)."""
    if torch.is_grad_enabled() and (Gs.requires_grad or hs.requires_grad):
        Ghs = torch.cat((Gs, hs.to(Gs.dtype).unsqueeze(2)), -1)
        Gs /= torch.max(torch.abs(Ghs), dim=2, keepdim=True)[0]
    else:
        with torch.no_grad():
            Ghs = torch.cat((Gs, hs.to(Gs.dtype).unsqueeze(2)), -1)
            Gs.div_(torch.max(torch.abs(Ghs), dim=2, keepdim=True)[0])


# qpth.qp.QPFunction.__init__'s keyword arguments that cbf_layer's solver_args may carry.  `verbose`
# is one of them, but the reference already passes it (QPFunction(verbose=0, **solver_args),
# diff_cbf_qp.py:139), so solver_args holding it is a duplicate keyword: TypeError there and here.
_QPFUNCTION_ARGS = ("eps", "notImprovedLim", "maxIter", "solver", "check_Q_spd")


class CBFQPLayer:

    def __init__(self, env, args, gamma_b=100, k_d=1.5, l_p=0.03, solver=_lib.SOLVER_ACTIVE_SET):
        """rcbf_sac/diff_cbf_qp.py:12-42 (same arguments and attributes).
        `solver` selects the fp64 QP algorithm: exact Goldfarb-Idnani active
        set (default) or the qpth-style primal-dual interior point."""
        self.device = torch.device("cuda" if getattr(args, "cuda", False) else "cpu")
        self.env = env
        self.u_min, self.u_max = self.get_control_bounds()
        self.gamma_b = gamma_b
        if self.env.dynamics_mode not in DYNAMICS_MODE:
            raise Exception("Dynamics mode not supported.")
        if self.env.dynamics_mode == "Unicycle":
            self.num_cbfs = len(env.hazards_locations)
            self.k_d = k_d
            self.l_p = l_p
        elif self.env.dynamics_mode == "SimulatedCars":
            self.num_cbfs = 2
        self.action_dim = env.action_space.shape[0]
        self.num_ineq_constraints = self.num_cbfs + 2 * self.action_dim
        self._prm = make_params(env, gamma_b, k_d, l_p, _lib.FORM_DIFF, solver)
        self.check_failures = True
        _lib.load()

    # -- diff_cbf_qp.py:44-79 ----------------------------------------------
    def get_safe_action(self, state_batch, action_batch, mean_pred_batch, sigma_batch):
        expand_dims = len(state_batch.shape) == 1
        if expand_dims:
            action_batch = action_batch.unsqueeze(0)
            state_batch = state_batch.unsqueeze(0)
            mean_pred_batch = mean_pred_batch.unsqueeze(0) if mean_pred_batch is not None else None
            sigma_batch = sigma_batch.unsqueeze(0) if sigma_batch is not None else None
        out_device = action_batch.device if torch.is_tensor(action_batch) else self.device
        dev = _dev()
        x = _f32(state_batch, dev)
        mu = _f32(mean_pred_batch, dev) if mean_pred_batch is not None else None
        sig = _f32(sigma_batch, dev) if sigma_batch is not None else None
        if torch.is_tensor(action_batch) and action_batch.requires_grad:
            u = action_batch.to(device=dev, dtype=torch.float32)
            if not u.is_contiguous():
                u = u.contiguous()
        else:
            u = _f32(action_batch, dev)
        self._check_shapes(x, u, mu, sig)
        final_action = safe_action_op(self, x, u, mu, sig)
        if final_action.device != out_device:
            final_action = final_action.to(out_device)
        return final_action if not expand_dims else final_action.squeeze(0)

    def _check_shapes(self, x, u, mu, sig):
        n_s = DYNAMICS_MODE[self.env.dynamics_mode]["n_s"]
        B = x.shape[0]
        if x.dim() != 2 or x.shape[1] != n_s or u.shape != (B, self.action_dim):
            raise ValueError(f"expected state (B,{n_s}) and action (B,{self.action_dim}), got "
                             f"{tuple(x.shape)} / {tuple(u.shape)}")
        for t in (mu, sig):
            if t is not None and t.shape != x.shape:
                raise ValueError("mean/sigma must have the state's shape")

    # -- diff_cbf_qp.py:146-379 --------------------------------------------
    def get_cbf_qp_constraints(self, state_batch, action_batch, mean_pred_batch, sigma_pred_batch):
        assert len(state_batch.shape) == 2 and len(action_batch.shape) == 2 and len(mean_pred_batch.shape) == 2 \
            and len(sigma_pred_batch.shape) == 2, (state_batch.shape, action_batch.shape)
        dev = _dev()
        x, u = _f32(state_batch, dev), _f32(action_batch, dev)
        mu, sig = _f32(mean_pred_batch, dev), _f32(sigma_pred_batch, dev)
        self._check_shapes(x, u, mu, sig)
        B, n, m = x.shape[0], self.action_dim + 1, self.num_ineq_constraints
        P = torch.empty(B, n, n, device=dev)
        q = torch.empty(B, n, device=dev)
        G = torch.empty(B, m, n, device=dev)
        h = torch.empty(B, m, device=dev)
        rc = _lib.load().rcbf_build(ctypes.byref(self._prm), B, _lib.ptr(x), _lib.ptr(u), _lib.ptr(mu),
                                    _lib.ptr(sig), _lib.ptr(P), _lib.ptr(q), _lib.ptr(G), _lib.ptr(h),
                                    _lib.stream_of(dev))
        _lib.check(rc, "rcbf_build")
        od = state_batch.device if torch.is_tensor(state_batch) else self.device
        return P.to(od), q.to(od), G.to(od), h.to(od)

    # -- diff_cbf_qp.py:81-109 ---------------------------------------------
    def solve_qp(self, Ps, qs, Gs, hs):
        """Row-normalise then solve; returns the solution without the slack.
        The kernel normalises and solves in one launch (rcbf_qp_solve_saved,
        normalize=1).  Like the reference (`Gs /= Ghs_norm`,
        diff_cbf_qp.py:103-105) the caller's Gs tensor is divided in place:
        without autograd history under no_grad, otherwise as the reference's
        own in-place op (a leaf that requires grad raises the same
        RuntimeError, a non-leaf records the division).  The solve reads a
        copy of the rows, so the inputs its backward saved are not the ones
        divided afterwards."""
        G_in = Gs.clone() if torch.is_tensor(Gs) else Gs
        sol = self._qp(Ps, qs, G_in, hs, normalize=True)
        if torch.is_tensor(Gs) and torch.is_tensor(hs):
            _divide_rows_in_place(Gs, hs)
        return sol[:, :-1]

    # -- diff_cbf_qp.py:111-144 --------------------------------------------
    def cbf_layer(self, Qs, ps, Gs, hs, As=None, bs=None, solver_args=None):
        """`solver_args` are qpth QPFunction's keyword arguments, as the
        reference passes them (diff_cbf_qp.py:132-139; solve_qp sends
        check_Q_spd, maxIter, notImprovedLim, eps, :107).  An unknown key
        raises TypeError, as QPFunction(**solver_args) does, and so does
        `verbose` (the reference already passes verbose=0, :139).  With the
        interior-point solver (solver=SOLVER_PDIPM) `maxIter` and `eps` set its
        iteration cap and stopping tolerance (notImprovedLim is the
        reference's 10); the exact solvers return the optimum whatever the
        tolerance, so they read none of them."""
        prm = self._solver_params(solver_args)
        if As is not None and As.numel() > 0:
            raise NotImplementedError("equality constraints are not used on this path (diff_cbf_qp.py:135-137)")
        return self._qp(Qs, ps, Gs, hs, normalize=False, prm=prm)

    def _solver_params(self, solver_args):
        if not solver_args:
            return self._prm
        for k in solver_args:
            if k == "verbose":  # QPFunction(verbose=0, **solver_args) (diff_cbf_qp.py:139)
                raise TypeError("QPFunction() got multiple values for keyword argument 'verbose'")
            if k not in _QPFUNCTION_ARGS:
                raise TypeError(f"QPFunction.__init__() got an unexpected keyword argument '{k}'")
        if self._prm.solver != _lib.SOLVER_PDIPM or ("maxIter" not in solver_args and "eps" not in solver_args):
            return self._prm
        prm = _lib.RcbfParams.from_buffer_copy(self._prm)
        if "maxIter" in solver_args:
            prm.max_iter = int(solver_args["maxIter"])
        if "eps" in solver_args:
            prm.eps = float(solver_args["eps"])
        return prm

    def _qp(self, Ps, qs, Gs, hs, normalize, prm=None):
        dev = _dev()
        G, h = _f32_keep_grad(Gs, dev), _f32_keep_grad(hs, dev)
        if G.dim() != 3 or h.shape != G.shape[:2]:
            raise ValueError(f"expected G (B,m,n) and h (B,m), got {tuple(G.shape)} / {tuple(h.shape)}")
        B, m, n = G.shape
        P = _f32_keep_grad(Ps, dev)
        if P.dim() == 2:  # qpth broadcasts an unbatched Q
            P = P.expand(B, n, n).contiguous()
        q = _f32_keep_grad(qs, dev) if qs is not None else None
        if q is not None and q.dim() == 1:
            q = q.expand(B, n).contiguous()
        if P.shape != (B, n, n) or (q is not None and q.shape != (B, n)):
            raise ValueError("P must be (B,n,n) and q (B,n)")
        z = _QP.apply(self, self._prm if prm is None else prm, bool(normalize), P, q, G, h)
        od = Gs.device if torch.is_tensor(Gs) else self.device
        return z.to(od)

    # -- diff_cbf_qp.py:381-395 --------------------------------------------
    def get_control_bounds(self):
        u_min = torch.tensor(self.env.safe_action_space.low).to(self.device)
        u_max = torch.tensor(self.env.safe_action_space.high).to(self.device)
        return u_min, u_max
