"""Device-resident environments (envs/simulated_cars_env.py, envs/unicycle_env.py).

* BatchedSimulatedCarsEnv / BatchedUnicycleEnv: B envs whose fp64 state lives
  in HBM; reset/step/safe_step/rollout are single HIP launches (rcbf_env_*,
  rcbf_safe_step, rcbf_safe_rollout) with auto-reset of finished envs.
* SimulatedCarsEnv / UnicycleEnv: the reference's single-env gym API
  (reset() -> obs, step(a) -> (obs, reward, done, info), seed/close/render,
  action_space/observation_space/safe_action_space, max_episode_steps, dt,
  dynamics_mode, kp/k_brake, hazards_*) on a B = 1 device env, so the
  reference's main.py loop runs unchanged.

Per-env state in HBM, component-pair-major (include/rcbf_hip.h) so every
component-pair access of a wavefront is one contiguous 1 KiB dwordx4 access:
x (n_s * B,) f64 holds env.state (`.state` is the (B, n_s) tensor); aux (B,) f64 = env.t (cars) or env.last_goal_dist (unicycle); step (B,)
i32 = env.episode_step; episode (B,) i32 = reset counter keying the
counter-based reset RNG (so the cars' N(0, 0.5) reset draw depends only on
(seed, global env index, episode) and is identical however the envs are
sharded over GPUs).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .params import make_params

# The optional CPython binding (csrc/rcbf_pyfast.cpp), bound by _lib.load() to
# the library ctypes loaded.  Tests set _fast = None to force the ctypes path.
_FAST_DEFAULT = object()
_fast = _FAST_DEFAULT


def _fast_binding():
    return _lib.fast() if _fast is _FAST_DEFAULT else _fast

try:  # keep gym's types when gym is installed (it is not in this image)
    import gym as _gym
    _EnvBase = _gym.Env
except Exception:  # pragma: no cover - exercised when gym is absent
    _gym = None
    _EnvBase = object


class Box:
    """Minimal gym.spaces.Box: float32 low/high/shape, sample/seed/contains."""

    def __init__(self, low, high, shape):
        self.shape = tuple(shape)
        self.low = np.full(self.shape, low, dtype=np.float32)
        self.high = np.full(self.shape, high, dtype=np.float32)
        self.dtype = np.float32
        self._rng = np.random.RandomState()

    def seed(self, s=None):
        self._rng = np.random.RandomState(s)
        return [s]

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(np.float32)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))


def _box(low, high, shape):
    if _gym is not None:
        return _gym.spaces.Box(low=low, high=high, shape=shape)
    return Box(low, high, shape)


class _EnvSpec:
    """Constants of one env family (the reference's __init__ attributes)."""

    def __init__(self, mode):
        self.dynamics_mode = mode
        if mode == "SimulatedCars":  # simulated_cars_env.py:17-26
            self.action_space = _box(-1.0, 1.0, (1,))
            self.safe_action_space = _box(-10.0, 10.0, (1,))
            self.observation_space = _box(-1e10, 1e10, (10,))
            self.max_episode_steps = 300
            self.dt = 0.02
            self.kp = 4.0
            self.k_brake = 20.0
            self.n_s, self.n_u, self.n_o = 10, 1, 10
        else:  # unicycle_env.py:17-34
            self.action_space = _box(-1.0, 1.0, (2,))
            self.safe_action_space = _box(-2.5, 2.5, (2,))
            self.observation_space = _box(-1e10, 1e10, (7,))
            self.bds = np.array([[-3., -3.], [3., 3.]])
            self.hazards_radius = 0.6
            self.hazards_locations = np.array([[0., 0.], [-1., 1.], [-1., -1.], [1., -1.], [1., 1.]]) * 1.5
            self.dt = 0.02
            self.max_episode_steps = 1000
            self.reward_goal = 1.0
            self.goal_size = 0.3
            self.goal_pos = np.array([2.5, 2.5])
            self.n_s, self.n_u, self.n_o = 3, 2, 7


def pairs_to_rows(xf, n_s, B):
    """(n_s*B,) component-pair-major buffer -> (B, n_s) rows."""
    P = n_s // 2
    rows = xf[:2 * P * B].view(P, B, 2).permute(1, 0, 2).reshape(B, 2 * P)
    if n_s % 2:
        rows = torch.cat([rows, xf[2 * P * B:].view(B, 1)], 1)
    return rows


def rows_to_pairs(rows):
    """(B, n_s) rows -> (n_s*B,) component-pair-major buffer."""
    B, n_s = rows.shape
    P = n_s // 2
    head = rows[:, :2 * P].reshape(B, P, 2).permute(1, 0, 2).reshape(-1)
    if n_s % 2:
        head = torch.cat([head, rows[:, n_s - 1].contiguous()])
    return head.contiguous()


class BatchedEnv:
    """B independent envs resident on one HIP device."""

    def __init__(self, mode, num_envs, device=None, seed=0, env_offset=0, hazards_locations=None):
        spec = _EnvSpec(mode)
        self.__dict__.update({k: v for k, v in spec.__dict__.items()})
        if hazards_locations is not None:
            self.hazards_locations = np.asarray(hazards_locations, np.float64).reshape(-1, 2)
        if not torch.cuda.is_available():
            raise RuntimeError("device envs need a HIP device (MI355X); there is no CPU fallback")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        self.seed_value = int(seed)
        self.env_offset = int(env_offset)  # global index of env 0 (sharding)
        B, d = self.num_envs, self.device
        self.x = torch.zeros(self.n_s * B, dtype=torch.float64, device=d)  # component-pair-major
        self.aux = torch.zeros(B, dtype=torch.float64, device=d)
        self.step_count = torch.zeros(B, dtype=torch.int32, device=d)
        self.episode = torch.zeros(B, dtype=torch.int32, device=d)
        self.obs = torch.zeros(B, self.n_o, dtype=torch.float32, device=d)
        self._prm_env = make_params(self, 1.0)
        self.fail_flag = torch.zeros(1, dtype=torch.int32, device=d)
        _lib.load()
        self.reset()

    @property
    def state(self):
        """(B, n_s) tensor of the env states (a copy out of the pair-major buffer)."""
        return pairs_to_rows(self.x, self.n_s, self.num_envs)

    def state_numpy(self):
        return self.state.cpu().numpy()

    def load_state(self, x=None, aux=None, step=None):
        """Overwrite the state of every env: x (B, n_s), aux (B,), step (B,)."""
        def dev(v, dt):
            v = v if isinstance(v, torch.Tensor) else np.asarray(v)
            return torch.as_tensor(v, device=self.device).to(dt)

        if x is not None:
            rows = dev(x, torch.float64)
            self.x.copy_(rows_to_pairs(rows.reshape(self.num_envs, self.n_s)))
        if aux is not None:
            self.aux.copy_(dev(aux, torch.float64).reshape(-1))
        if step is not None:
            self.step_count.copy_(dev(step, torch.int32).reshape(-1))

    def _rng_seed(self):
        return self.seed_value & 0xFFFFFFFFFFFFFFFF

    def _stream(self):
        return _lib.stream_of(self.device)

    def reset(self, noise=None, mask=None):
        """Reset all envs (or those with mask != 0).  `noise` (B,) f64 injects
        the cars' N(0,0.5) velocity draw (simulated_cars_env.py:120)."""
        nz = None
        if noise is not None:
            nz = torch.as_tensor(noise, dtype=torch.float64, device=self.device).reshape(-1).contiguous()
        mk = None
        if mask is not None:
            mk = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        rc = _lib.load().rcbf_env_reset(ctypes.byref(self._prm_env), self.num_envs, _lib.ptr(mk), _lib.ptr(nz),
                                        self._rng_seed(), self.env_offset, _lib.ptr(self.x), _lib.ptr(self.aux),
                                        _lib.ptr(self.step_count), _lib.ptr(self.episode), _lib.ptr(self.obs),
                                        self._stream())
        _lib.check(rc, "rcbf_env_reset")
        return self.obs

    def step(self, action, auto_reset=True, obs64=False):
        """Batched env.step: action (B, n_u) f32 or f64 (reward dtype follows
        the action like the reference).  Returns obs (B,n_o) f32, reward (B,)
        f64, done (B,) bool, info dict(cost (B,) f64, goal_met (B,) bool[, obs64])."""
        a = torch.as_tensor(action, device=self.device)
        if a.dtype not in (torch.float32, torch.float64):
            a = a.to(torch.float32)
        a = a.reshape(self.num_envs, self.n_u).contiguous()
        B, d = self.num_envs, self.device
        reward = torch.empty(B, dtype=torch.float64, device=d)
        cost = torch.empty(B, dtype=torch.float64, device=d)
        done = torch.empty(B, dtype=torch.uint8, device=d)
        goal = torch.empty(B, dtype=torch.uint8, device=d)
        o64 = torch.empty(B, self.n_o, dtype=torch.float64, device=d) if obs64 else None
        rc = _lib.load().rcbf_env_step(ctypes.byref(self._prm_env), B, _lib.ptr(self.x), _lib.ptr(self.aux),
                                       _lib.ptr(self.step_count), _lib.ptr(self.episode), _lib.ptr(a),
                                       int(a.dtype == torch.float64), _lib.ptr(o64), _lib.ptr(self.obs),
                                       _lib.ptr(reward), _lib.ptr(cost), _lib.ptr(done), _lib.ptr(goal),
                                       int(auto_reset), self._rng_seed(), self.env_offset, self._stream())
        _lib.check(rc, "rcbf_env_step")
        info = {"cost": cost, "goal_met": goal.bool()}
        if obs64:
            info["obs64"] = o64
        return self.obs, reward, done.bool(), info

    def _prior_arg(self, t, name):
        """mean / sigma as the kernel reads them: (B, n_s) fp32, contiguous, on
        this env's device (None -> the in-kernel prior)."""
        if t is None:
            return None
        B, d = self.num_envs, self.device
        if not (torch.is_tensor(t) and t.dtype == torch.float32 and t.is_contiguous() and t.device == d):
            t = torch.as_tensor(t, dtype=torch.float32, device=d).contiguous()
        if t.shape != (B, self.n_s):
            raise ValueError(f"{name} must be ({B}, {self.n_s}), got {tuple(t.shape)}")
        return t

    # output dimensions of the disturbance prediction the CBF rows read, in
    # the column layout of rcbf_safe_step_cols: cars sigma[:, 5], [:, 7],
    # [:, 9] (no mean, diff_cbf_qp.py:298-299); unicycle all three of each
    PRIOR_COLS = {"SimulatedCars": (5, 7, 9), "Unicycle": (0, 1, 2)}

    def _prior_cols_arg(self, t, name):
        """mean / sigma in column layout: (len(PRIOR_COLS), B) fp32."""
        if t is None:
            return None
        B, d = self.num_envs, self.device
        if not (torch.is_tensor(t) and t.dtype == torch.float32 and t.is_contiguous() and t.device == d):
            t = torch.as_tensor(t, dtype=torch.float32, device=d).contiguous()
        nc = len(self.PRIOR_COLS[self.dynamics_mode])
        if t.shape != (nc, B):
            raise ValueError(f"{name} (column layout) must be ({nc}, {B}), got {tuple(t.shape)}")
        return t

    def safe_step(self, u_rl, layer, mean=None, sigma=None, auto_reset=True, outputs=None, prior_layout="rows"):
        """The fused hot path (rcbf_safe_step): state -> get_state(obs32) ->
        CBFQPLayer.get_safe_action(state, u_rl, mean, sigma) -> env.step.
        mean/sigma None -> the DynamicsModel prior in-kernel.  `outputs`
        (from make_outputs) avoids per-call allocation; failures accumulate
        in self.fail_flag (check with check_failures()).
        The ctypes argument list is cached per (layer, outputs tensors,
        auto_reset): an eager call then costs one data_ptr per changing
        input, so the host keeps pace with the ~4 us kernel."""
        o = outputs if outputs is not None else self.make_outputs()
        u = self._u_arg(u_rl)
        if prior_layout == "cols":
            # (len(PRIOR_COLS), B) columns (rcbf_safe_step_cols; e.g. GPDisturbanceModel.predict_cols)
            if mean is not None and self.dynamics_mode == "SimulatedCars":
                raise ValueError("the cars CBF rows read no mean (diff_cbf_qp.py:298-299): pass mean=None")
            mean, sigma = self._prior_cols_arg(mean, "mean"), self._prior_cols_arg(sigma, "sigma")
            args = self._step_args(layer, o, auto_reset)
            rc = _lib.load().rcbf_safe_step_cols(
                ctypes.byref(layer._prm), self.num_envs, *[a or None for a in args[2:6]], u.data_ptr(),
                None if mean is None else mean.data_ptr(), None if sigma is None else sigma.data_ptr(),
                *[a or None for a in args[9:17]], *args[17:20],
                torch._C._cuda_getCurrentRawStream(self.device.index) or None)
            _lib.check(rc, "rcbf_safe_step_cols")
            return self.obs, o["reward"], o["done"], o
        if prior_layout != "rows":
            raise ValueError(f"prior_layout must be 'rows' or 'cols', got {prior_layout!r}")
        mean, sigma = self._prior_arg(mean, "mean"), self._prior_arg(sigma, "sigma")
        args = self._step_args(layer, o, auto_reset)
        args[6] = u.data_ptr()
        args[7] = 0 if mean is None else mean.data_ptr()
        args[8] = 0 if sigma is None else sigma.data_ptr()
        args[20] = torch._C._cuda_getCurrentRawStream(self.device.index)
        fast = _fast_binding()
        if fast is not None:  # CPython binding (csrc/rcbf_pyfast.cpp): ~1 us instead of ~4 us through ctypes
            rc = fast.safe_step(*args)
        else:
            rc = _lib.load().rcbf_safe_step(ctypes.byref(layer._prm), self.num_envs, *[a or None for a in args[2:17]],
                                            *args[17:20], args[20] or None)
        _lib.check(rc, "rcbf_safe_step")
        return self.obs, o["reward"], o["done"], o

    def safe_step_seq(self, u_rl_seq, layer, mean=None, sigma=None, auto_reset=True, outputs=None, steps=None,
                      prior_layout="rows"):
        """`steps` fused safe steps (default len(u_rl_seq)) issued from ONE host
        call (rcbf_safe_step_seq, or rcbf_safe_step_seq_cols for
        prior_layout="cols"): step j uses u_rl_seq[j % len(u_rl_seq)], each
        (B, n_u) f32 on this device.  Every step is its own launch of the
        fused kernel, exactly as `steps` calls of safe_step; the outputs hold
        the last step's values."""
        o = outputs if outputs is not None else self.make_outputs()
        us = [self._u_arg(u) for u in u_rl_seq]
        if not us:
            raise ValueError("u_rl_seq is empty")
        K = len(us) if steps is None else int(steps)
        if prior_layout not in ("rows", "cols"):
            raise ValueError(f"prior_layout must be 'rows' or 'cols', got {prior_layout!r}")
        cols = prior_layout == "cols"
        if cols:
            if mean is not None and self.dynamics_mode == "SimulatedCars":
                raise ValueError("the cars CBF rows read no mean (diff_cbf_qp.py:298-299): pass mean=None")
            mean, sigma = self._prior_cols_arg(mean, "mean"), self._prior_cols_arg(sigma, "sigma")
        else:
            mean, sigma = self._prior_arg(mean, "mean"), self._prior_arg(sigma, "sigma")
        a = list(self._step_args(layer, o, auto_reset))
        stream = torch._C._cuda_getCurrentRawStream(self.device.index)
        ptrs = [t.data_ptr() for t in us]
        fast = None if cols else _fast_binding()
        tail = a[9:17] + a[17:20]
        if cols:
            arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
            rc = _lib.load().rcbf_safe_step_seq_cols(ctypes.byref(layer._prm), self.num_envs, K,
                                                     *[v or None for v in a[2:6]], arr, len(ptrs),
                                                     None if mean is None else mean.data_ptr(),
                                                     None if sigma is None else sigma.data_ptr(),
                                                     *[v or None for v in a[9:17]], *a[17:20], stream or None)
            _lib.check(rc, "rcbf_safe_step_seq_cols")
            return self.obs, o["reward"], o["done"], o
        if fast is not None:
            rc = fast.safe_step_seq(a[0], a[1], K, *a[2:6], ptrs, 0 if mean is None else mean.data_ptr(),
                                    0 if sigma is None else sigma.data_ptr(), *tail, stream)
        else:
            arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
            rc = _lib.load().rcbf_safe_step_seq(ctypes.byref(layer._prm), self.num_envs, K,
                                                *[v or None for v in a[2:6]], arr, len(ptrs),
                                                None if mean is None else mean.data_ptr(),
                                                None if sigma is None else sigma.data_ptr(),
                                                *[v or None for v in a[9:17]], *a[17:20], stream or None)
        _lib.check(rc, "rcbf_safe_step_seq")
        return self.obs, o["reward"], o["done"], o

    def safe_step_span(self, u_rl, layer, span, mean=None, sigma=None, auto_reset=True, outputs=None,
                       prior_layout="rows"):
        """safe_step through the measurement entry point rcbf_safe_step_span:
        the same step, plus each wave's start / end chip-clock stamps and
        shader-clock stamps in `span` ((ceil(B / 64), 4) int64 on this
        device: realtime start, end, memtime start, end).  bench.py only."""
        o = outputs if outputs is not None else self.make_outputs()
        u = self._u_arg(u_rl)
        cols = prior_layout == "cols"
        if cols:
            mean, sigma = self._prior_cols_arg(mean, "mean"), self._prior_cols_arg(sigma, "sigma")
        else:
            mean, sigma = self._prior_arg(mean, "mean"), self._prior_arg(sigma, "sigma")
        nw = (self.num_envs + 63) // 64
        if not (torch.is_tensor(span) and span.dtype == torch.int64 and span.device == self.device
                and span.is_contiguous() and span.numel() >= 4 * nw):
            raise ValueError(f"span must be a contiguous int64 tensor of >= {4 * nw} entries on {self.device}")
        a = self._step_args(layer, o, auto_reset)
        rc = _lib.load().rcbf_safe_step_span(
            ctypes.byref(layer._prm), self.num_envs, *[v or None for v in a[2:6]], u.data_ptr(),
            None if mean is None else mean.data_ptr(), None if sigma is None else sigma.data_ptr(), int(cols),
            *[v or None for v in a[9:17]], *a[17:20], span.data_ptr(),
            torch._C._cuda_getCurrentRawStream(self.device.index) or None)
        _lib.check(rc, "rcbf_safe_step_span")
        return self.obs, o["reward"], o["done"], o

    def _u_arg(self, u_rl):
        B, d = self.num_envs, self.device
        u = u_rl if (torch.is_tensor(u_rl) and u_rl.dtype == torch.float32 and u_rl.is_contiguous()
                     and u_rl.device == d) else torch.as_tensor(u_rl, dtype=torch.float32, device=d).contiguous()
        if u.shape != (B, self.n_u):
            raise ValueError(f"u_rl must be ({B}, {self.n_u}), got {tuple(u.shape)}")
        return u

    def _check_layer(self, layer):
        """The fused kernel runs the env physics with the LAYER's params: they
        must describe this env (mode, hazards, gains), or it would index the
        state buffers with the wrong dimension."""
        p, q = layer._prm, self._prm_env
        same = (p.mode == q.mode and p.num_hazards == q.num_hazards and p.kp == q.kp and p.k_brake == q.k_brake
                and p.hazards_radius == q.hazards_radius
                and all(p.hazards_xy[k] == q.hazards_xy[k] for k in range(2 * q.num_hazards)))
        if not same:
            raise ValueError("the CBF layer was built for a different env (dynamics mode, hazards or gains differ)")

    def _check_outputs(self, o):
        B, d = self.num_envs, self.device
        want = {"u": ((B, self.n_u), torch.float32), "reward": ((B,), torch.float32),
                "cost": ((B,), torch.float32), "done": ((B,), torch.uint8), "goal_met": ((B,), torch.uint8)}
        for k, (shape, dt) in want.items():
            t = o.get(k)
            if t is None and k == "goal_met":
                continue
            if not (torch.is_tensor(t) and tuple(t.shape) == shape and t.dtype == dt and t.device == d
                    and t.is_contiguous()):
                raise ValueError(f"outputs[{k!r}] must be a contiguous {dt} tensor of shape {shape} on {d} "
                                 "(use make_outputs())")

    def _step_args(self, layer, o, auto_reset):
        """The argument list of rcbf_safe_step (u_rl/mean/sigma/stream slots
        filled per call), cached per (layer params, outputs, auto_reset, RNG
        seed, shard offset); layer and outputs are validated when an entry is
        built, so the check stays off the per-step path."""
        key = (id(layer), id(layer._prm), bool(auto_reset), self._rng_seed(), self.env_offset,
               tuple(map(id, o.values())))
        ent = getattr(self, "_ss_cache", {}).get(key)
        if ent is None or ent[0] is not layer or ent[1] is not o or ent[4] is not layer._prm:
            self._check_layer(layer)
            self._check_outputs(o)
            self._ss_cache = {}

            def p(t):
                return 0 if t is None else t.data_ptr()
            # the cars env never meets a goal (info['goal_met'] is always False,
            # simulated_cars_env.py:85): its goal_met output is zero-filled once
            # here and the kernel is not asked to write it every step
            gm = o.get("goal_met")
            if gm is not None and self.dynamics_mode == "SimulatedCars":
                gm.zero_()
                gm = None
            args = [ctypes.addressof(layer._prm), self.num_envs, p(self.x), p(self.aux), p(self.step_count),
                    p(self.episode), 0, 0, 0, p(self.obs), p(o["u"]), p(o["reward"]), p(o["cost"]), p(o["done"]),
                    p(gm), 0, p(self.fail_flag), int(auto_reset), self._rng_seed(), self.env_offset, 0]
            ent = self._ss_cache[key] = (layer, o, args, [t for t in o.values() if t is not None], layer._prm)
        return ent[2]

    def make_outputs(self):
        B, d = self.num_envs, self.device
        return {"u": torch.empty(B, self.n_u, dtype=torch.float32, device=d),
                "reward": torch.empty(B, dtype=torch.float32, device=d),
                "cost": torch.empty(B, dtype=torch.float32, device=d),
                "done": torch.empty(B, dtype=torch.uint8, device=d),
                "goal_met": torch.empty(B, dtype=torch.uint8, device=d)}

    def rollout(self, u_rl_seq, layer):
        """K fused safe steps in one launch (rcbf_safe_rollout) from a
        pre-sampled u_rl (K, B, n_u) f32, prior mean/sigma, auto-reset.
        Returns per-env reward sum, cost sum and episodes finished."""
        B, d = self.num_envs, self.device
        u = torch.as_tensor(u_rl_seq, dtype=torch.float32, device=d).contiguous()
        K = u.shape[0]
        rs = torch.empty(B, dtype=torch.float32, device=d)
        cs = torch.empty(B, dtype=torch.float32, device=d)
        nd = torch.empty(B, dtype=torch.int32, device=d)
        rc = _lib.load().rcbf_safe_rollout(ctypes.byref(layer._prm), B, K, _lib.ptr(self.x), _lib.ptr(self.aux),
                                           _lib.ptr(self.step_count), _lib.ptr(self.episode), _lib.ptr(u),
                                           _lib.ptr(self.obs), _lib.ptr(rs), _lib.ptr(cs), _lib.ptr(nd),
                                           _lib.ptr(self.fail_flag), self._rng_seed(), self.env_offset, self._stream())
        _lib.check(rc, "rcbf_safe_rollout")
        return rs, cs, nd

    def check_failures(self):
        bits = int(self.fail_flag.item())
        if bits:
            self.fail_flag.zero_()
            raise Exception("QP Failed to solve")


class BatchedSimulatedCarsEnv(BatchedEnv):
    def __init__(self, num_envs, device=None, seed=0, env_offset=0):
        super().__init__("SimulatedCars", num_envs, device, seed, env_offset)


class BatchedUnicycleEnv(BatchedEnv):
    def __init__(self, num_envs, device=None, seed=0, env_offset=0, hazards_locations=None):
        super().__init__("Unicycle", num_envs, device, seed, env_offset, hazards_locations)


class _SingleEnv(_EnvBase):
    """The reference's single-env gym surface on a B = 1 device env."""
    metadata = {"render.modes": ["human"]}

    def __init__(self, mode):
        spec = _EnvSpec(mode)
        self.__dict__.update(spec.__dict__)
        self._np_rng = np.random
        self._b = BatchedEnv(mode, 1, seed=0)
        self.viewer = None
        self.reset()

    # env.state / env.t / env.episode_step / env.last_goal_dist as numpy views
    @property
    def state(self):
        return self._b.x.cpu().numpy().copy()  # B = 1: the buffer is the state row

    @state.setter
    def state(self, v):
        self._b.x.copy_(torch.as_tensor(np.asarray(v, np.float64).reshape(-1), device=self._b.device))

    @property
    def episode_step(self):
        return int(self._b.step_count[0].item())

    @episode_step.setter
    def episode_step(self, v):
        self._b.step_count[0] = int(v)

    def seed(self, s=None):
        self.action_space.seed(s)
        return [s]

    def close(self):
        pass

    @property
    def unwrapped(self):
        return self

    def _host_io(self):
        """Pinned, device-coherent host buffers the step kernel reads the
        action from and writes its results to (rcbf_host_alloc), plus the
        cached argument list of rcbf_env_step_sync."""
        io = getattr(self, "_io", None)
        if io is not None:
            return io
        lib, b, n_o = _lib.load(), self._b, self.n_o
        # packed outputs | pad | completion word (at 8 (n_o + 2) + 8) | f32 action (2) | f64 action (2)
        nbytes = 8 * (n_o + 2) + 16 + 16 + 16
        p = ctypes.c_void_p()
        _lib.check(lib.rcbf_host_alloc(nbytes + 16, ctypes.byref(p)), "rcbf_host_alloc")
        base = (p.value + 15) & ~15
        act = 8 * (n_o + 2) + 16
        io = {"raw": p.value, "base": base,
              "pk": np.ctypeslib.as_array((ctypes.c_double * (n_o + 2)).from_address(base)),
              "flags": np.ctypeslib.as_array((ctypes.c_uint8 * 2).from_address(base + 8 * (n_o + 2))),
              "a32": np.ctypeslib.as_array((ctypes.c_float * 2).from_address(base + act)),
              "a64": np.ctypeslib.as_array((ctypes.c_double * 2).from_address(base + act + 16)),
              "a32p": base + act, "a64p": base + act + 16,
              "args": [ctypes.addressof(b._prm_env), 1, b.x.data_ptr(), b.aux.data_ptr(), b.step_count.data_ptr(),
                       b.episode.data_ptr(), 0, 0, base, 0, b._rng_seed(), b.env_offset, 0]}
        self._io = io
        return io

    def __del__(self):
        io = getattr(self, "_io", None)
        if io is not None and _lib is not None:
            try:
                _lib.load().rcbf_host_free(io["raw"])
            except Exception:
                pass

    def step(self, action):
        """One env step in ONE host call (rcbf_env_step_sync): the kernel
        reads the action from pinned host memory, steps the device-resident
        env and writes obs (fp64), reward, cost, done and goal_met straight
        into pinned host memory; the call returns once the stream is done."""
        a = np.asarray(action)
        if a.dtype not in (np.float32, np.float64):
            a = a.astype(np.float32)
        f64 = a.dtype == np.float64
        io = self._host_io()
        n_o = self.n_o
        if f64:
            io["a64"][:self.n_u] = a.reshape(-1)
        else:
            io["a32"][:self.n_u] = a.reshape(-1)
        args = io["args"]
        args[6] = io["a64p"] if f64 else io["a32p"]
        args[7] = int(f64)
        args[12] = torch._C._cuda_getCurrentRawStream(self._b.device.index)
        fast = _fast_binding()
        if fast is not None:
            rc = fast.env_step_sync(*args)
        else:
            rc = _lib.load().rcbf_env_step_sync(ctypes.byref(self._b._prm_env), 1, *args[2:10], args[10], args[11],
                                                args[12] or None)
        _lib.check(rc, "rcbf_env_step_sync")
        pk = io["pk"]
        obs = pk[:n_o].copy()
        r = np.float64(pk[n_o]) if f64 else np.float32(pk[n_o])
        return obs, r, bool(io["flags"][0]), self._info_host(float(pk[n_o + 1]), bool(io["flags"][1]))

    def render(self, mode="human", close=False):
        print("Ep_step = {}, \tState = {}".format(self.episode_step, self.state))


class SimulatedCarsEnv(_SingleEnv):
    """envs/simulated_cars_env.py:6-158 on the device env."""

    def __init__(self):
        super().__init__("SimulatedCars")

    @property
    def t(self):
        return float(self._b.aux[0].item())

    @t.setter
    def t(self, v):
        self._b.aux[0] = float(v)

    def reset(self):
        # the N(0, 0.5) draw comes from the global numpy RNG like the reference (:120)
        noise = np.array([self._np_rng.normal(0, 0.5)])
        self._b.reset(noise=noise)
        return self._get_obs()

    def _get_obs(self):
        s = self.state
        o = s.copy()
        o[::2] /= 100.0
        o[1::2] /= 30.0
        return o

    def _info_host(self, cost, goal):
        return {"cost": cost, "goal_met": False}


class UnicycleEnv(_SingleEnv):
    """envs/unicycle_env.py:8-280 on the device env (render is out of scope)."""

    def __init__(self):
        super().__init__("Unicycle")

    @property
    def last_goal_dist(self):
        return float(self._b.aux[0].item())

    @last_goal_dist.setter
    def last_goal_dist(self, v):
        self._b.aux[0] = float(v)

    def _goal_dist(self):
        return float(np.linalg.norm(self.goal_pos - self.state[:2]))

    def reset(self):
        self._b.reset()
        return self.get_obs()

    def get_obs(self):
        s = self.state
        rel = self.goal_pos - s[:2]
        gd = np.linalg.norm(rel)
        c, sn = np.cos(s[2]), np.sin(s[2])
        v = np.matmul(rel, np.array([[c, -sn], [sn, c]]))
        v /= np.sqrt(np.sum(np.square(v))) + 0.001
        return np.array([s[0], s[1], c, sn, v[0], v[1], np.exp(-gd)])

    def goal_met(self):
        return np.linalg.norm(self.state[:2] - self.goal_pos) <= self.goal_size

    def _info_host(self, c, goal):
        out = {}
        if goal:
            out["goal_met"] = True
        if c > 0:
            out["cost"] = c
        return out
