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
* Predict (the per-step hot path): rcbf_gp_predict, the GP posterior mean
  and predictive std on the device (csrc/rcbf_gp.hip) from [R | alpha],
  where R R^T ~ (K + nI)^-1.  The reference predicts under
  gpytorch.settings.fast_pred_var() (LOVE, gp_model.py:97-99): gpytorch's
  root_inv_decomposition takes the Cholesky inverse root L^-T (the exact
  posterior) up to max_cholesky_size = 800 training points and, above that,
  a Lanczos inverse root of rank <= max_root_decomposition_size = 100 from one
  random start vector (torch.randn).  love_rank(N) restates that choice and
  love_inv_root restates the Lanczos root (linear_operator's lanczos_tridiag
  with full reorthogonalisation, then the Ritz decomposition), in fp64 on the
  device; the oracle restates it again in numpy (oracle.love_inv_root).  The
  start vectors come from a torch.Generator of their own (DynamicsModel
  seeds it from its seed, so drawing them leaves torch's global CPU stream,
  which seeded user code consumes, unchanged; gpytorch itself draws from the
  global stream) and are kept (`love_init`), so a fit is reproducible.  Parity
  against gpytorch itself is unpinned (not installed; its start vector is
  random anyway).  The Lanczos runs in fp64 here; gpytorch's GPs are fp32.
* The mean's alpha = (K + nI)^-1 y: by default gpytorch's eval-mode solve
  (cg_mean_solve: Cholesky up to 800 points, linear_cg at the eval tolerance
  0.01 above, preconditioned from 2000 points by a rank-15 pivoted Cholesky;
  restated in fp64 from linear_operator's published algorithm, oracle
  gp_mean_solve).  That CG stops at a 1 % relative residual, not at the exact
  solve: on the GPU tests' fits at N = 3000 its mean sits 1-4 % of max|mean|
  from the exact solve, on fits under the reference's own priors ~4e-4
  (profiles/r06/gp_mean_cg_gap.json).  mean_solve="exact" keeps the exact
  solve.  Parity with gpytorch: unpinned.
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib

_PAD_N = 32
_PAD_C = 128


MAX_CHOLESKY_SIZE = 800  # gpytorch.settings.max_cholesky_size default
MAX_ROOT_SIZE = 100      # gpytorch.settings.max_root_decomposition_size default


def love_rank(N):
    """The variance factor gpytorch's fast_pred_var builds for N training
    points: None = the Cholesky inverse root (exact) at N <= 800, else a
    Lanczos inverse root of size min(100, N)."""
    return None if N <= MAX_CHOLESKY_SIZE else min(MAX_ROOT_SIZE, N)


def lanczos_tridiag(C, init_vec, max_iter, tol=1e-5):
    """linear_operator.utils.lanczos.lanczos_tridiag for one SPD matrix C
    (N, N) and one start vector (N,) (torch, C's device and dtype): Lanczos
    with classical Gram-Schmidt reorthogonalisation against all earlier
    vectors, up to 10 extra passes while an inner product exceeds tol; stops
    when beta <= 1e-6 or the extra passes fail.  Returns Q (N, k), T (k, k)."""
    N = C.shape[0]
    num_iter = min(int(max_iter), N)
    Q = torch.zeros(num_iter, N, dtype=C.dtype, device=C.device)
    T = torch.zeros(num_iter, num_iter, dtype=C.dtype, device=C.device)
    v = init_vec.to(dtype=C.dtype, device=C.device)
    q0 = v / torch.linalg.vector_norm(v)
    Q[0] = q0
    r = C @ q0
    a0 = q0 @ r
    r = r - a0 * q0
    b0 = torch.linalg.vector_norm(r)
    T[0, 0] = a0
    if num_iter > 1:
        T[0, 1] = b0
        T[1, 0] = b0
        Q[1] = r / b0
    k = 0
    for k in range(1, num_iter):
        r = C @ Q[k] - Q[k - 1] * T[k, k - 1]
        ac = Q[k] @ r
        T[k, k] = ac
        if k + 1 < num_iter:
            r = r - ac * Q[k]
            Qk = Q[:k + 1]
            r = r - Qk.t() @ (Qk @ r)
            bc = torch.linalg.vector_norm(r)
            r = r / bc
            T[k, k + 1] = bc
            T[k + 1, k] = bc
            could = False
            for _ in range(10):
                if not bool(((Qk @ r) > tol).any()):
                    could = True
                    break
                r = r - Qk.t() @ (Qk @ r)
                r = r / torch.linalg.vector_norm(r)
            Q[k + 1] = r
            if float(bc.abs()) <= 1e-6 or not could:
                break
    n = k + 1
    return Q[:n].t(), T[:n, :n]


def love_inv_root(C, init_vec, max_iter):
    """LOVE's inverse root (linear_operator RootDecomposition with
    inverse=True): R = Q V diag(lam)^-1/2 from the Lanczos T = V diag(lam)
    V^T, negative Ritz values masked (their columns zero), so
    R R^T = Q T^-1 Q^T ~ C^-1.  Returns R (N, k)."""
    Q, T = lanczos_tridiag(C, init_vec, max_iter)
    lam, V = torch.linalg.eigh(T)
    keep = lam >= 0
    V = V * keep[None, :].to(V.dtype)
    lam = torch.where(keep, lam, torch.ones_like(lam))
    return (Q @ V) / torch.sqrt(lam)[None, :]


CG_EVAL_TOLERANCE = 0.01    # gpytorch.settings.eval_cg_tolerance
CG_MAX_ITER = 1000          # settings.max_cg_iterations
CG_MIN_ITER = 10            # linear_cg stops no earlier than k = min(10, max_iter - 1)
CG_MIN_PRECOND_SIZE = 2000  # settings.min_preconditioning_size
CG_PRECOND_RANK = 15        # settings.max_preconditioner_size
PRECOND_TOLERANCE = 1e-3    # settings.preconditioner_tolerance


def pivoted_cholesky(K, rank, error_tol=PRECOND_TOLERANCE):
    """linear_operator's pivoted_cholesky (torch, K's device and dtype): greedy
    max-diagonal pivots, at most `rank` steps, stopping once the remaining
    diagonal's L1 norm / max(diag K) <= error_tol.  Returns L (N, m)."""
    N = K.shape[0]
    diag = torch.diagonal(K).clone()
    perm = torch.arange(N, device=K.device)
    rank = min(rank, N)
    L = torch.zeros(rank, N, dtype=K.dtype, device=K.device)
    orig = float(diag.max())
    err = float(diag.abs().sum()) / orig
    m = 0
    while m == 0 or (m < rank and err > error_tol):
        i = m + int(torch.argmax(diag[perm[m:]]))
        pm_old = perm[m].clone()
        perm[m] = perm[i]
        perm[i] = pm_old
        pm = int(perm[m])
        L[m, pm] = torch.sqrt(diag[pm])
        if m + 1 < N:
            pi = perm[m + 1:]
            new = K[pm, pi].clone()
            if m > 0:
                new = new - (L[:m, pm][:, None] * L[:m, pi]).sum(0)
            new = new / L[m, pm]
            L[m, pi] = new
            diag[pi] = diag[pi] - new * new
            err = float(diag[pi].abs().sum()) / orig
        m += 1
    return L[:m].t().contiguous()


def linear_cg(matmul, rhs, precond=None, tol=CG_EVAL_TOLERANCE, max_iter=CG_MAX_ITER, eps=1e-10,
              stop_updating_after=1e-10):
    """linear_operator.utils.linear_cg for one right-hand side (torch): unit-
    norm rhs, x0 = 0, safe divisions, stop at the first k >= min(10,
    max_iter - 1) with |r| < tol.  Returns (x, iterations)."""
    P = precond if precond is not None else (lambda r: r)
    nrm = torch.linalg.vector_norm(rhs)
    if float(nrm) < eps:
        nrm = torch.ones_like(nrm)
    b = rhs / nrm
    x = torch.zeros_like(b)
    r = b.clone()
    if float(torch.linalg.vector_norm(r)) < stop_updating_after:
        return x * nrm, 0
    z = P(r)
    p = z.clone()
    rz = z @ r
    k = 0
    for k in range(max_iter):
        Ap = matmul(p)
        a = p @ Ap
        a = torch.zeros_like(a) if float(a) < eps else rz / a
        r = r - a * Ap
        z = P(r)
        x = x + a * p
        rz_new = r @ z
        beta = torch.zeros_like(rz) if float(rz) < eps else rz_new / rz
        rz = rz_new
        p = z + beta * p
        rn = float(torch.linalg.vector_norm(r))
        if rn < stop_updating_after:
            break
        if k >= min(CG_MIN_ITER, max_iter - 1) and rn < tol:
            break
    return x * nrm, k + 1


def cg_mean_solve(K, noise, y):
    """gpytorch's eval-mode mean_cache (K + noise I)^-1 y (oracle
    gp_mean_solve): Cholesky up to 800 points, else linear_cg on K + noise I,
    from 2000 points with the pivoted-Cholesky preconditioner of K in its
    Woodbury form v -> (v - Q Q^T v) / noise, [L; sqrt(noise) I] = Q R (NaNs in
    L: unpreconditioned, as linear_operator falls back).  K without the noise;
    torch, K's device and dtype."""
    N = K.shape[0]
    C = K + noise * torch.eye(N, dtype=K.dtype, device=K.device)
    if N <= MAX_CHOLESKY_SIZE:
        return torch.cholesky_solve(y[:, None], torch.linalg.cholesky(C))[:, 0]
    precond = None
    if N >= CG_MIN_PRECOND_SIZE:
        Lp = pivoted_cholesky(K, CG_PRECOND_RANK)
        if not bool(torch.isnan(Lp).any()):
            k = Lp.shape[1]
            Q, _ = torch.linalg.qr(torch.cat([Lp, math.sqrt(noise) * torch.eye(k, dtype=K.dtype, device=K.device)], 0))
            Q = Q[:N]

            def precond(v):
                return (v - Q @ (Q.t() @ v)) / noise
    return linear_cg(lambda v: C @ v, y, precond)[0]


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

    def __init__(self, train_x, train_y, hyper, device=None, rank=None, love_init=None, mean_solve="exact",
                 love_generator=None, raw_train=False):
        """train_x, train_y: (N, n_s) raw history (dynamics.py:307-312);
        hyper: per dim (lengthscale, outputscale, noise).  rank None: the
        exact posterior (Cholesky inverse root); rank r: LOVE's Lanczos
        inverse root of size <= r (love_rank(N) gives gpytorch's choice) from
        the start vectors love_init (n_s, N) (default: torch.randn from
        love_generator, a torch.Generator, or else the global CPU generator, as
        gpytorch draws its own).  mean_solve: "exact" (Cholesky) or "cg"
        (gpytorch's eval-mode solve, cg_mean_solve).  raw_train: condition on
        the raw training data instead of the normalised data (what the
        reference's load_disturbance_models does, dynamics.py:401-403); the
        queries are normalised and the outputs rescaled either way."""
        if mean_solve not in ("exact", "cg"):
            raise ValueError(f"mean_solve must be 'exact' or 'cg', got {mean_solve!r}")
        self.mean_solve = mean_solve
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        tx = np.asarray(train_x, np.float64)
        ty = np.asarray(train_y, np.float64)
        N, n_s = tx.shape
        self.n_s, self.N, self.device = n_s, N, dev
        self.rank = None if rank is None else int(rank)
        self.love_init = None
        if self.rank is not None:
            self.love_init = (torch.randn(n_s, N, dtype=torch.float64, generator=love_generator) if love_init is None else
                              torch.as_tensor(np.asarray(love_init, np.float64)).reshape(n_s, N).clone())
        x_std = tx.std(axis=0)
        y_std = ty.std(axis=0)
        # dynamics.py:315-318: training data normalised by std + 1e-8, as fp32 tensors
        self.raw_train = bool(raw_train)
        xn = torch.as_tensor(tx if raw_train else tx / (x_std + 1e-8), dtype=torch.float32, device=dev)
        yn = torch.as_tensor(ty if raw_train else ty / (y_std + 1e-8), dtype=torch.float32, device=dev)
        self.hyper = [tuple(map(float, h)) for h in hyper]
        N_pad = -(-N // _PAD_N) * _PAD_N
        x64 = xn.double()
        d2 = torch.cdist(x64, x64).pow(2)
        eye = torch.eye(N, dtype=torch.float64, device=dev)
        Rs, alphas = [], []
        for i, (ls, os_, nz) in enumerate(self.hyper):
            C = os_ * torch.exp(-0.5 * d2 / (ls * ls)) + nz * eye
            y = yn[:, i].double()
            L = torch.linalg.cholesky(C)
            if mean_solve == "cg":  # gpytorch's eval-mode mean solve
                alpha = cg_mean_solve(C - nz * eye, nz, y)
            else:
                alpha = torch.cholesky_solve(y[:, None], L)[:, 0]
            if self.rank is None:  # exact: C^-1 = L^-T L^-1, R = L^-T
                R = torch.linalg.solve_triangular(L, eye, upper=False).t()
            else:                  # LOVE: Lanczos inverse root of size <= rank (gp_model.py:97-99)
                R = love_inv_root(C, self.love_init[i], self.rank)
            Rs.append(R)
            alphas.append(alpha)
        self.alpha = torch.stack(alphas)  # (n_s, N) f64: the mean weights (dynamics.py:371-380 mean_cache)
        # one factor width for all GPs (a Lanczos run may stop early): zero columns add nothing to |k R|^2
        self.r = max(R.shape[1] for R in Rs)
        C_pad = -(-(self.r + 1) // _PAD_C) * _PAD_C
        xt = torch.zeros(n_s, N_pad, n_s, dtype=torch.float32, device=dev)
        Rt = torch.zeros(n_s, N_pad, C_pad, dtype=torch.float32, device=dev)
        for i, (ls, os_, nz) in enumerate(self.hyper):
            xt[i, :N] = (xn * np.float32(1.0 / (math.sqrt(2.0) * ls)))
            Rt[i, :N, :Rs[i].shape[1]] = Rs[i].float()
            Rt[i, :N, self.r] = alphas[i].float()
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
        flags = _lib.GP_RT_UPPER if self.rank is None else 0
        self._m = _lib.RcbfGpModel(n_s, N, N_pad, self.r, C_pad, flags, *(t.data_ptr() for t in (
            self.xt, self.tn2, self.Rt, self.x_std, self.inv_sl, self.outscale, self.noise, self.y_scale)))
        # one workspace per stream: the B <= 8 GEMV's arrival counters live in it, so two calls in flight on
        # two streams must not share one (include/rcbf_hip.h rcbf_gp_workspace_floats); zero-filled when made
        self._ws = {}

    def _workspace(self, B):
        """(workspace, stream) for a call of B queries on the current stream."""
        lib = _lib.load()
        stream = _lib.stream_of(self.device)
        need = int(lib.rcbf_gp_workspace_floats(ctypes.byref(self._m), B))
        key = stream.value or 0
        ws = self._ws.get(key)
        if ws is None or ws.numel() < need:
            ws = self._ws[key] = torch.zeros(need, dtype=torch.float32, device=self.device)  # counters start at zero
        return ws, stream

    def check_failures(self):
        """Synchronously check every workspace's GEMV hand-off
        (rcbf_gp_workspace_check): raises RuntimeError if a call found a
        non-zero arrival counter (its outputs were not valid); the counters are
        zeroed either way, so the next call is clean."""
        lib = _lib.load()
        bad = []
        for key, ws in self._ws.items():
            rc = lib.rcbf_gp_workspace_check(ctypes.byref(self._m), _lib.ptr(ws), ctypes.c_void_p(key) if key else None)
            if rc == 1006:
                bad.append(key)
            elif rc:
                _lib.check(rc, "rcbf_gp_workspace_check")
        if bad:
            raise RuntimeError("GP posterior: a GEMV call found a non-zero arrival counter (workspace not zero-filled, "
                               "an aborted call, or two calls sharing one workspace); its outputs were invalid, the "
                               "counters are reset")

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
        ws, stream = self._workspace(B)
        rc = lib.rcbf_gp_predict(ctypes.byref(self._m), B, _lib.ptr(x), _lib.ptr(mean), _lib.ptr(std), _lib.ptr(ws),
                                 stream)
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
        ws, stream = self._workspace(B)
        rc = lib.rcbf_gp_predict_cols(ctypes.byref(self._m), B, _lib.ptr(x), _lib.ptr(mr), _lib.ptr(sr), carr,
                                      len(cols), _lib.ptr(mc), _lib.ptr(sc), _lib.ptr(ws), stream)
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


def fit(train_x, train_y, prior_std, training_iter=70, device=None, rank=None, love_init=None, mean_solve="exact",
        love_generator=None):
    """DynamicsModel.fit_gp_model (dynamics.py:296-340) -> GPDisturbanceModel
    (rank, mean_solve, love_generator: see GPDisturbanceModel; DynamicsModel
    passes love_rank(N), its gp_mean and its own generator)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    tx = np.asarray(train_x, np.float64)
    ty = np.asarray(train_y, np.float64)
    xn = torch.as_tensor(tx / (tx.std(axis=0) + 1e-8), dtype=torch.float32, device=dev).double()
    yn = torch.as_tensor(ty / (ty.std(axis=0) + 1e-8), dtype=torch.float32, device=dev).double()
    hyper = [train_hyperparameters(xn, yn[:, i], float(prior_std[i]), training_iter) for i in range(tx.shape[1])]
    return GPDisturbanceModel(tx, ty, hyper, device=dev, rank=rank, love_init=love_init, mean_solve=mean_solve,
                              love_generator=love_generator)
