"""Device-resident ReplayMemory (rcbf_sac/replay_memory.py:5-38, SURVEY 8f
row 4).

The reference keeps a Python list of tuples, pushes in a Python loop
(batch_push, "TODO: Optimize This", :23-29) and samples with random.sample +
np.stack (:31-35).  Here the transitions live in HBM as one ring of packed
fp64 records [state | action | reward | next_state | mask | t | next_t]:
batch_push is one scatter launch (rcbf_ring_scatter_f64) and sample one
gather launch (rcbf_gather_rows_f64) on indices drawn without replacement
(uniform, like random.sample; numpy's Generator instead of Python's random,
so the sampled indices differ from the reference's stream).

sample() returns numpy arrays like the reference (mask as float64, t/next_t
NaN when they were pushed as None); sample_tensors() keeps them on the device
for the SAC update.
"""
import ctypes

import numpy as np
import torch

from . import _lib


class ReplayMemory:

    def __init__(self, capacity, seed, device=None):
        self.capacity = int(capacity)
        self.position = 0
        self._size = 0
        self._rng = np.random.default_rng(seed)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._ring = None
        self._dims = None  # (n_s, n_u)

    # -- layout -------------------------------------------------------------
    def _width(self):
        n_s, n_u = self._dims
        return 2 * n_s + n_u + 4

    def _pack(self, state, action, reward, next_state, mask, t, next_t):
        def col(v, n):
            if v is None:
                return torch.full((n, 1), float("nan"), dtype=torch.float64, device=self.device)
            v = v if torch.is_tensor(v) else torch.as_tensor(np.asarray(v, dtype=np.float64))
            return v.to(device=self.device, dtype=torch.float64).reshape(n, -1)

        state = state if torch.is_tensor(state) else np.asarray(state, dtype=np.float64)
        n = state.shape[0]
        st = col(state, n)
        act = col(action, n)
        if self._dims is None:
            self._dims = (st.shape[1], act.shape[1])
            self._ring = torch.empty(self.capacity, self._width(), dtype=torch.float64, device=self.device)
        if (st.shape[1], act.shape[1]) != self._dims:
            raise ValueError(f"transition shapes {(st.shape[1], act.shape[1])} != {self._dims}")
        rec = torch.cat([st, act, col(reward, n), col(next_state, n), col(mask, n), col(t, n), col(next_t, n)], 1)
        return rec.contiguous()

    # -- reference API ------------------------------------------------------
    def push(self, state, action, reward, next_state, mask, t=None, next_t=None):
        def one(v):
            return None if v is None else (v.unsqueeze(0) if torch.is_tensor(v) else np.asarray(v)[None])
        self.batch_push(one(state), one(action), one(reward), one(next_state), one(mask), one(t), one(next_t))

    def batch_push(self, state_batch, action_batch, reward_batch, next_state_batch, mask_batch, t_batch=None,
                   next_t_batch=None):
        if t_batch is None or next_t_batch is None:  # the reference drops both unless both are given (:25-29)
            t_batch = next_t_batch = None
        rec = self._pack(state_batch, action_batch, reward_batch, next_state_batch, mask_batch, t_batch,
                         next_t_batch)
        n = rec.shape[0]
        if n == 0:
            return
        if n > self.capacity:  # the sequential pushes leave only the last `capacity` records
            self.position = (self.position + n - self.capacity) % self.capacity
            rec = rec[n - self.capacity:].contiguous()
            n = self.capacity
        rc = _lib.load().rcbf_ring_scatter_f64(_lib.ptr(self._ring), self.capacity, rec.shape[1], self.position,
                                               _lib.ptr(rec), n, _lib.stream_of(self.device))
        _lib.check(rc, "rcbf_ring_scatter_f64")
        self.position = (self.position + n) % self.capacity
        self._size = min(self._size + n, self.capacity)

    def sample_tensors(self, batch_size):
        """(state, action, reward, next_state, mask, t, next_t) device tensors."""
        if batch_size > self._size or batch_size < 0:
            raise ValueError("Sample larger than population or is negative")
        idx = torch.as_tensor(self._rng.choice(self._size, batch_size, replace=False).astype(np.int64),
                              device=self.device)
        out = torch.empty(batch_size, self._width(), dtype=torch.float64, device=self.device)
        rc = _lib.load().rcbf_gather_rows_f64(_lib.ptr(out), _lib.ptr(self._ring), out.shape[1], _lib.ptr(idx),
                                              batch_size, _lib.stream_of(self.device))
        _lib.check(rc, "rcbf_gather_rows_f64")
        n_s, n_u = self._dims
        o = 0
        parts = []
        for w in (n_s, n_u, 1, n_s, 1, 1, 1):
            parts.append(out[:, o:o + w])
            o += w
        s, a, r, ns, m, t, nt = parts
        return s, a, r[:, 0], ns, m[:, 0], t[:, 0], nt[:, 0]

    def sample(self, batch_size):
        return tuple(v.cpu().numpy() for v in self.sample_tensors(batch_size))

    def __len__(self):
        return self._size
