"""GP disturbance model: rcbf_sac/gp_model.py +
DynamicsModel.fit_gp_model / predict_disturbance (rcbf_sac/dynamics.py:296-390).

* Fit (host-side set-up, once per gp_model_size/10 transitions): one exact GP
  per state dimension with the reference model -- ZeroMean, ScaleKernel(RBF)
  with NormalPrior(1e5, 1e-5) on the lengthscale and NormalPrior(prior_std +
  1e-6, 1e-5) on the outputscale, GaussianLikelihood (noise > 1e-4) -- whose
  hyperparameters are trained like gpytorch's ExactGP: Adam(lr 0.1) on
  -(log N(y; 0, K + nI) + log priors) / N for `training_iter` steps, with
  gpytorch's softplus parametrisation and initial values (gp_model.py:14-21,
  55-78).  gpytorch itself is not installed here, so this is a restatement of
  its published algorithm (fp64 on the device instead of its fp32), parity
  unpinned against gpytorch; tests pin it to the numpy oracle.
* Predict (the per-step hot path): rcbf_gp_predict, the exact GP posterior
  mean and predictive std on the fp32 MFMA (csrc/rcbf_gp.hip).  gpytorch's
  fast_pred_var (LOVE, gp_model.py:97) approximates this variance; `rank` < N
  gives the analogous low-rank variance (top-r eigenpairs of K + nI).
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib

_PAD_N = 32
_PAD_C = 128


def _softplus(x):
    return torch.nn.functional.softplus(x)


def _inv_softplus(v):
    v = torch.as_tensor(v, dtype=torch.float64)
    return v + torch.log(-torch.expm1(-v))  # gpytorch.utils.transforms.inv_softplus


def train_hyperparameters(x, y, prior_std, training_iter=70, lr=0.1):
    """GPyDisturbanceEstimator.train (gp_model.py:55-78) for one GP.
    x (N, D) and y (N,) fp64 device tensors (normalised as fit_gp_model does).
    Returns (lengthscale, outputscale, noise) as Python floats."""
    dev = x.device
    N = x.shape[0]
    d2 = torch.cdist(x, x).pow(2)
    raw = torch.stack([torch.zeros((), dtype=torch.float64),                     # likelihood.raw_noise
                       _inv_softplus(1e5),                                       # raw_lengthscale
                       _inv_softplus(prior_std + 1e-6)]).to(dev).requires_grad_(True)
    opt = torch.optim.Adam([raw], lr=lr)
    eye = torch.eye(N, dtype=torch.float64, device=dev)
    ls_loc, os_loc, sc = 1e5, prior_std + 1e-6, 1e-5
    for _ in range(training_iter):
        opt.zero_grad()
        noise = 1e-4 + _softplus(raw[0])
        ls = _softplus(raw[1])
        os_ = _softplus(raw[2])
        C = os_ * torch.exp(-0.5 * d2 / (ls * ls)) + noise * eye
        L = torch.linalg.cholesky(C)
        a = torch.cholesky_solve(y[:, None], L)[:, 0]
        logp = -0.5 * (y @ a) - torch.log(torch.diagonal(L)).sum() - 0.5 * N * math.log(2 * math.pi)
        lprior = (-(ls - ls_loc) ** 2 / (2 * sc * sc) - math.log(sc) - 0.5 * math.log(2 * math.pi)
                  - (os_ - os_loc) ** 2 / (2 * sc * sc) - math.log(sc) - 0.5 * math.log(2 * math.pi))
        loss = -(logp + lprior) / N
        loss.backward()
        opt.step()
    with torch.no_grad():
        return float(_softplus(raw[1])), float(_softplus(raw[2])), float(1e-4 + _softplus(raw[0]))


class GPDisturbanceModel:
    """The n_s fitted GPs of a DynamicsModel, resident on the device in the
    layout rcbf_gp_predict reads (include/rcbf_hip.h rcbf_gp_model)."""

    def __init__(self, train_x, train_y, hyper, device=None, rank=None):
        """train_x, train_y: (N, n_s) raw history (dynamics.py:307-312);
        hyper: per dim (lengthscale, outputscale, noise)."""
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        tx = np.asarray(train_x, np.float64)
        ty = np.asarray(train_y, np.float64)
        N, n_s = tx.shape
        self.n_s, self.N, self.device = n_s, N, dev
        self.r = N if rank is None else int(min(rank, N))
        x_std = tx.std(axis=0)
        y_std = ty.std(axis=0)
        # dynamics.py:315-318: training data normalised by std + 1e-8, as fp32 tensors
        xn = torch.as_tensor(tx / (x_std + 1e-8), dtype=torch.float32, device=dev)
        yn = torch.as_tensor(ty / (y_std + 1e-8), dtype=torch.float32, device=dev)
        self.hyper = [tuple(map(float, h)) for h in hyper]
        N_pad = -(-N // _PAD_N) * _PAD_N
        C_pad = -(-(self.r + 1) // _PAD_C) * _PAD_C
        xt = torch.zeros(n_s, N_pad, n_s, dtype=torch.float32, device=dev)
        Rt = torch.zeros(n_s, N_pad, C_pad, dtype=torch.float32, device=dev)
        x64 = xn.double()
        d2 = torch.cdist(x64, x64).pow(2)
        eye = torch.eye(N, dtype=torch.float64, device=dev)
        for i, (ls, os_, nz) in enumerate(self.hyper):
            isl = 1.0 / (math.sqrt(2.0) * ls)
            xt[i, :N] = (xn * np.float32(isl))
            C = os_ * torch.exp(-0.5 * d2 / (ls * ls)) + nz * eye
            y = yn[:, i].double()
            if self.r == N:  # exact: C^-1 = L^-T L^-1, R = L^-T
                L = torch.linalg.cholesky(C)
                Linv = torch.linalg.solve_triangular(L, eye, upper=False)
                R = Linv.t()
                alpha = torch.cholesky_solve(y[:, None], L)[:, 0]
            else:            # top-r eigenpairs of C (the subspace LOVE's Lanczos captures)
                lam, U = torch.linalg.eigh(C)
                R = U[:, -self.r:] / torch.sqrt(lam[-self.r:])[None]
                alpha = torch.linalg.solve(C, y)
            Rt[i, :N, :self.r] = R.float()
            Rt[i, :N, self.r] = alpha.float()
        self.xt = xt.contiguous()
        self.tn2 = (xt.double() ** 2).sum(-1).float().contiguous()
        # lane-interleave each 128-column block: physical 4 l + c <- logical 32 c + l
        n_cb = C_pad // _PAD_C
        self.Rt = Rt.view(n_s, N_pad, n_cb, 4, 32).permute(0, 1, 2, 4, 3).contiguous().view(n_s, N_pad, C_pad)
        self.x_std = torch.as_tensor(x_std, dtype=torch.float64, device=dev)
        self.inv_sl = torch.tensor([1.0 / (math.sqrt(2.0) * h[0]) for h in self.hyper], dtype=torch.float32, device=dev)
        self.outscale = torch.tensor([h[1] for h in self.hyper], dtype=torch.float32, device=dev)
        self.noise = torch.tensor([h[2] for h in self.hyper], dtype=torch.float32, device=dev)
        self.y_scale = torch.as_tensor(y_std + 1e-8, dtype=torch.float32, device=dev)
        # exact: R = L^-T is upper triangular, so the kernels skip the zero rows of each column block
        flags = _lib.GP_RT_UPPER if self.r == N else 0
        self._m = _lib.RcbfGpModel(n_s, N, N_pad, self.r, C_pad, flags, *(t.data_ptr() for t in (
            self.xt, self.tn2, self.Rt, self.x_std, self.inv_sl, self.outscale, self.noise, self.y_scale)))
        self._ws = torch.empty(0, dtype=torch.float32, device=dev)

    def logical_Rt(self):
        """(n_s, N_pad, C_pad) [R | alpha | 0] in logical column order."""
        n_s, N_pad, C_pad = self.Rt.shape
        return self.Rt.view(n_s, N_pad, C_pad // _PAD_C, 32, 4).permute(0, 1, 2, 4, 3).reshape(n_s, N_pad, C_pad)

    def predict(self, x):
        """x (B, n_s) float32 device tensor -> (mean, std) (B, n_s) float32."""
        lib = _lib.load()
        x = x.to(device=self.device, dtype=torch.float32).contiguous()
        B = x.shape[0]
        mean = torch.empty(B, self.n_s, dtype=torch.float32, device=self.device)
        std = torch.empty_like(mean)
        need = int(lib.rcbf_gp_workspace_floats(ctypes.byref(self._m), B))
        if self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.float32, device=self.device)
        rc = lib.rcbf_gp_predict(ctypes.byref(self._m), B, _lib.ptr(x), _lib.ptr(mean), _lib.ptr(std),
                                 _lib.ptr(self._ws), _lib.stream_of(self.device))
        _lib.check(rc, "rcbf_gp_predict")
        return mean, std

    def predict_cols(self, x, cols, mean=True, rows=False):
        """The same posterior in the COLUMN layout the fused step reads
        (rcbf_gp_predict_cols -> rcbf_safe_step_cols): (mean_cols, std_cols),
        each (len(cols), B) float32 (mean_cols None when mean=False, e.g. the
        cars std columns (5, 7, 9), whose rows ignore the mean); with rows=True
        also the (B, n_s) rows: (mean_cols, std_cols, mean, std)."""
        lib = _lib.load()
        x = x.to(device=self.device, dtype=torch.float32).contiguous()
        B = x.shape[0]
        cols = [int(c) for c in cols]
        carr = (ctypes.c_int32 * max(1, len(cols)))(*cols)
        mc = torch.empty(len(cols), B, dtype=torch.float32, device=self.device) if mean else None
        sc = torch.empty(len(cols), B, dtype=torch.float32, device=self.device)
        mr = torch.empty(B, self.n_s, dtype=torch.float32, device=self.device) if rows else None
        sr = torch.empty_like(mr) if rows else None
        need = int(lib.rcbf_gp_workspace_floats(ctypes.byref(self._m), B))
        if self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.float32, device=self.device)
        rc = lib.rcbf_gp_predict_cols(ctypes.byref(self._m), B, _lib.ptr(x), _lib.ptr(mr), _lib.ptr(sr), carr,
                                      len(cols), _lib.ptr(mc), _lib.ptr(sc), _lib.ptr(self._ws),
                                      _lib.stream_of(self.device))
        _lib.check(rc, "rcbf_gp_predict_cols")
        return (mc, sc, mr, sr) if rows else (mc, sc)

    def flops_per_query(self):
        """Algorithmic MFMA flops per query row of the k(x, X) [R | alpha]
        product: 2 N C_pad per GP dense; with the upper-triangular factor
        (exact posterior) column block cb only meets training rows below
        128 (cb + 1), so 2 * 128 * sum_cb min(N, 128 (cb + 1)) per GP."""
        n_cb = self._m.C_pad // _PAD_C
        if self._m.flags & _lib.GP_RT_UPPER:
            k = sum(min(self.N, _PAD_C * (cb + 1)) for cb in range(n_cb))
            return 2 * _PAD_C * k * self.n_s
        return 2 * self.N * self._m.C_pad * self.n_s


def fit(train_x, train_y, prior_std, training_iter=70, device=None, rank=None):
    """DynamicsModel.fit_gp_model (dynamics.py:296-340) -> GPDisturbanceModel."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    tx = np.asarray(train_x, np.float64)
    ty = np.asarray(train_y, np.float64)
    xn = torch.as_tensor(tx / (tx.std(axis=0) + 1e-8), dtype=torch.float32, device=dev).double()
    yn = torch.as_tensor(ty / (ty.std(axis=0) + 1e-8), dtype=torch.float32, device=dev).double()
    hyper = [train_hyperparameters(xn, yn[:, i], float(prior_std[i]), training_iter) for i in range(tx.shape[1])]
    return GPDisturbanceModel(tx, ty, hyper, device=dev, rank=rank)
