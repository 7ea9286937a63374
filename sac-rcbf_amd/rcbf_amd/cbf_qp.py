"""Drop-in `CascadeCBFLayer` (rcbf_sac/cbf_qp.py:5-358) on the HIP kernels.

get_u_safe builds the fp64 rows, normalises them and solves the QP exactly
(Goldfarb-Idnani, the algorithm of the quadprog call at cbf_qp.py:276) in one
launch of rcbf_cascade_u_safe.  It also accepts a batch (leading axis).
The reference's per-call print of the quadprog result (:278) is not kept;
its slack-violation warning (:283-284) is: any row whose slack |epsilon|
exceeds 0.1 prints the reference's message (get_u_safe and solve_qp).
"""
import ctypes
import threading
import weakref

import numpy as np
import torch

from . import _lib
from .dynamics import DYNAMICS_MODE
from .params import make_params


_SYNC_MAX_B = 256  # rcbf_cascade_u_safe_sync: one workgroup


def _warn_slack(eps):
    """cbf_qp.py:283-284: the reference's warning when the QP needed a slack
    |epsilon| > 0.1 (one line per such row)."""
    for e in np.asarray(eps, np.float64).reshape(-1):
        if np.abs(e) > 1e-1:
            print('CBF indicates constraint violation might occur. epsilon = {}'.format(e))


class CascadeCBFLayer:

    def __init__(self, env, gamma_b=100, k_d=1.5, l_p=0.03, solver=_lib.SOLVER_ACTIVE_SET):
        self.env = env
        self.u_min, self.u_max = self.get_control_bounds()
        self.gamma_b = gamma_b
        self.k_d = k_d
        self.l_p = l_p
        if self.env.dynamics_mode not in DYNAMICS_MODE:
            raise Exception("Dynamics mode not supported.")
        self._prm = make_params(env, gamma_b, k_d, l_p, _lib.FORM_CASCADE, solver)
        _lib.load()

    def get_u_safe(self, u_nom, s, mean_pred, sigma):
        """cbf_qp.py:29-53: u_safe such that env.step(u_nom + u_safe) is safe.
        Up to 256 samples (the reference's loop calls it on one): the inputs
        go into a pinned host block the kernel reads in place and the call
        returns on its completion word (rcbf_cascade_u_safe_sync) -- no copy
        and no stream synchronisation; larger batches go through device
        tensors (rcbf_cascade_u_safe)."""
        if not torch.cuda.is_available():
            raise RuntimeError("CascadeCBFLayer needs a HIP device (MI355X); there is no CPU fallback")
        un = np.asarray(u_nom, np.float64)
        single = un.ndim == 1
        if np.atleast_2d(un).shape[0] <= _SYNC_MAX_B:
            return self._get_u_safe_sync(un, s, mean_pred, sigma, single)
        dev = torch.device("cuda", torch.cuda.current_device())

        def d(a):
            return torch.as_tensor(np.atleast_2d(np.asarray(a, np.float64)), device=dev).contiguous()

        U, X, M, S = d(un), d(s), d(mean_pred), d(sigma)
        B = X.shape[0]
        out = torch.empty(B, U.shape[1], dtype=torch.float64, device=dev)
        eps = torch.empty(B, dtype=torch.float64, device=dev)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        rc = _lib.load().rcbf_cascade_u_safe(ctypes.byref(self._prm), B, _lib.ptr(U), _lib.ptr(X), _lib.ptr(M),
                                             _lib.ptr(S), _lib.ptr(out), None, _lib.ptr(flag), _lib.ptr(eps),
                                             _lib.stream_of(dev))
        _lib.check(rc, "rcbf_cascade_u_safe")
        if int(flag.item()):
            raise ValueError("constraints are inconsistent, no solution")  # quadprog's ValueError (:279-281)
        res = out.cpu().numpy()
        self.last_eps = eps.cpu().numpy()
        _warn_slack(self.last_eps)
        return res[0] if single else res

    def _get_u_safe_sync(self, un, s, mean_pred, sigma, single):
        U = np.atleast_2d(un)
        X = np.atleast_2d(np.asarray(s, np.float64))
        B, n_u = U.shape
        n_s = X.shape[1]
        dims = DYNAMICS_MODE[self.env.dynamics_mode]
        if X.shape[0] != B or n_s != dims["n_s"] or n_u != dims["n_u"]:
            raise ValueError(f"expected u_nom (B, {dims['n_u']}) and state (B, {dims['n_s']}), got {U.shape} / {X.shape}")
        st = self._staging(B, n_s, n_u)
        st["u"][:B * n_u] = U.reshape(-1)
        st["x"][:B * n_s] = X.reshape(-1)
        st["m"][:B * n_s] = np.atleast_2d(np.asarray(mean_pred, np.float64)).reshape(-1)
        st["s"][:B * n_s] = np.atleast_2d(np.asarray(sigma, np.float64)).reshape(-1)
        st["seq"] = (st["seq"] + 1) & 0xFFFFFFFF or 1
        dev = torch.cuda.current_device()
        rc = _lib.load().rcbf_cascade_u_safe_sync(ctypes.byref(self._prm), B, st["pu"], st["px"], st["pm"], st["ps"],
                                                  st["po"], st["pst"], st["pe"], st["pw"], st["seq"],
                                                  _lib.stream_of(dev))
        _lib.check(rc, "rcbf_cascade_u_safe_sync")
        if (st["status"][:B] != _lib.QP_OK).any():
            raise ValueError("constraints are inconsistent, no solution")  # quadprog's ValueError (:279-281)
        res = st["o"][:B * n_u].reshape(B, n_u).copy()
        self.last_eps = st["e"][:B].copy()
        _warn_slack(self.last_eps)
        return res[0] if single else res

    def _staging(self, B, n_s, n_u):
        """A pinned host block (rcbf_host_alloc) of _SYNC_MAX_B samples: u_nom,
        state, mean, sigma, u_safe, epsilon (f64), status (i32), the completion
        word; numpy views over it.  One block per calling thread: two threads
        calling get_u_safe on one layer at once must not share a completion
        word."""
        stages = self.__dict__.setdefault("_stages", {})
        tid = threading.get_ident()
        st = stages.get(tid)
        if st is not None:
            return st
        cap = _SYNC_MAX_B
        sizes = [("u", cap * n_u * 8), ("x", cap * n_s * 8), ("m", cap * n_s * 8), ("s", cap * n_s * 8),
                 ("o", cap * n_u * 8), ("e", cap * 8), ("status", cap * 4), ("w", 64)]
        total = sum(-(-b // 64) * 64 for _, b in sizes)
        ptr = ctypes.c_void_p()
        _lib.check(_lib.load().rcbf_host_alloc(total, ctypes.byref(ptr)), "rcbf_host_alloc")
        st, off = {"base": ptr.value, "seq": 0}, 0
        for name, b in sizes:
            a = ptr.value + off
            st["p" + ("st" if name == "status" else name)] = a
            if name == "status":
                st[name] = np.ctypeslib.as_array((ctypes.c_int32 * cap).from_address(a))
            elif name != "w":
                st[name] = np.ctypeslib.as_array((ctypes.c_double * (b // 8)).from_address(a))
            off += -(-b // 64) * 64
        ctypes.c_uint32.from_address(st["pw"]).value = 0
        stages[tid] = st
        st["fin"] = weakref.finalize(self, _lib.load().rcbf_host_free, ptr.value)
        return st

    def get_cbf_qp_constraints(self, u_nom, state, mean_pred, sigma_pred):
        """cbf_qp.py:55-240 (fp64), single sample or batch."""
        un = np.asarray(u_nom, np.float64)
        single = un.ndim == 1
        dev = torch.device("cuda", torch.cuda.current_device())

        def d(a):
            return torch.as_tensor(np.atleast_2d(np.asarray(a, np.float64)), device=dev).contiguous()

        U, X, M, S = d(un), d(state), d(mean_pred), d(sigma_pred)
        B = X.shape[0]
        n = U.shape[1] + 1
        m = (len(self.env.hazards_locations) if self.env.dynamics_mode == "Unicycle" else 2) + 2 * U.shape[1]
        P = torch.empty(B, n, n, dtype=torch.float64, device=dev)
        q = torch.empty(B, n, dtype=torch.float64, device=dev)
        G = torch.empty(B, m, n, dtype=torch.float64, device=dev)
        h = torch.empty(B, m, dtype=torch.float64, device=dev)
        rc = _lib.load().rcbf_build_f64(ctypes.byref(self._prm), B, _lib.ptr(X), _lib.ptr(U), _lib.ptr(M),
                                        _lib.ptr(S), _lib.ptr(P), _lib.ptr(q), _lib.ptr(G), _lib.ptr(h),
                                        _lib.stream_of(dev))
        _lib.check(rc, "rcbf_build_f64")
        P, q, G, h = (t.cpu().numpy() for t in (P, q, G, h))
        if single:
            return P[0], q[0], G[0], h[0]
        return P, q, G, h

    def solve_qp(self, P, q, G, h):
        """cbf_qp.py:242-286: normalise the rows of [G h] (G in place, like the
        reference's `G /= Gh_norm`), solve min 1/2 z'Pz + q'z s.t. Gz <= h
        exactly in fp64 (rcbf_qp_solve_f64, Goldfarb-Idnani as quadprog) and
        return z without the slack.  Infeasible -> quadprog's ValueError."""
        if not torch.cuda.is_available():
            raise RuntimeError("CascadeCBFLayer needs a HIP device (MI355X); there is no CPU fallback")
        Gh = np.concatenate((G, np.expand_dims(h, 1)), 1)
        Gh_norm = np.expand_dims(np.max(np.abs(Gh), axis=1), axis=1)
        G /= Gh_norm  # the caller's G, in place as :272
        h = h / Gh_norm.squeeze(-1)
        dev = torch.device("cuda", torch.cuda.current_device())
        m, n = np.shape(G)

        def d(a):
            return torch.as_tensor(np.asarray(a, np.float64).reshape(1, -1), device=dev).contiguous()

        Pd, qd, Gd, hd = d(P), d(q), d(G), d(h)
        z = torch.empty(1, n, dtype=torch.float64, device=dev)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        rc = _lib.load().rcbf_qp_solve_f64(ctypes.byref(self._prm), 1, n, m, _lib.ptr(Pd), _lib.ptr(qd), _lib.ptr(Gd),
                                           _lib.ptr(hd), 0, _lib.ptr(z), None, None, _lib.ptr(flag),
                                           _lib.stream_of(dev))
        _lib.check(rc, "rcbf_qp_solve_f64")
        if int(flag.item()):
            raise ValueError("constraints are inconsistent, no solution")
        zh = z[0].cpu().numpy()
        _warn_slack(zh[-1:])
        return zh[:-1]

    def get_cbfs(self, hazards_locations, hazards_radius):
        """cbf_qp.py:288-323: (get_h, get_dhdx) of the hazard CBFs
        h_j(s) = 1/2 (||p(s) - o_j||^2 - (r + 0.07)^2) on the look-ahead output
        p(s) (unicycle) or the state itself."""
        hz = np.array(hazards_locations)
        r = hazards_radius + 0.07

        def out(state):
            if self.env.dynamics_mode == "Unicycle":
                return np.array([state[0] + self.l_p * np.cos(state[2]), state[1] + self.l_p * np.sin(state[2])])
            return state

        def get_h(state):
            return 0.5 * (np.sum((out(state) - hz) ** 2, axis=1) - r ** 2)

        def get_dhdx(state):
            return out(state) - hz

        return get_h, get_dhdx

    def get_control_bounds(self):
        return self.env.safe_action_space.low, self.env.safe_action_space.high

    def get_min_h_val(self, state):
        """cbf_qp.py:341-358."""
        get_h, _ = self.get_cbfs(self.env.hazards_locations, self.env.hazards_radius)
        return np.min(get_h(state))
