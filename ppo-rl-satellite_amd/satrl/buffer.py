"""Transition storage.

* ``ReplayBuffer``  -- drop-in for replaybuffer.py:3-38 (flat, host numpy,
  float64, ``store`` at ``count % batch_size``, ``numpy_to_tensor`` -> f32).
* ``RolloutBuffer`` -- the engine's device-resident time-major buffer
  [T, N] for N parallel envs (HBM): obs is kept T+1 times (obs[t+1] is the
  post-reset observation where done[t]; V(s') of a done step is multiplied
  by (1 - dw) = 0 in the reference's GAE, so the terminal obs is not needed).
"""
from __future__ import annotations

import numpy as np
import torch


class ReplayBuffer:
    """replaybuffer.py:3-38."""

    def __init__(self, args):
        self.state_dim = args.state_dim
        self.action_dim = args.action_dim
        self.batch_size = args.batch_size
        self.s = np.zeros((args.batch_size, args.state_dim))
        self.a = np.zeros((args.batch_size, args.action_dim))
        self.a_logprob = np.zeros((args.batch_size, args.action_dim))
        self.r = np.zeros((args.batch_size, 1))
        self.s_ = np.zeros((args.batch_size, args.state_dim))
        self.dw = np.zeros((args.batch_size, 1))
        self.done = np.zeros((args.batch_size, 1))
        self.count = 0

    def store(self, s, a, a_logprob, r, s_, dw, done):
        index = self.count % self.batch_size
        self.s[index] = s
        self.a[index] = a
        self.a_logprob[index] = a_logprob
        self.r[index] = r
        self.s_[index] = s_
        self.dw[index] = dw
        self.done[index] = done
        self.count += 1

    def numpy_to_tensor(self):
        f = torch.float
        return (torch.tensor(self.s, dtype=f), torch.tensor(self.a, dtype=f), torch.tensor(self.a_logprob, dtype=f),
                torch.tensor(self.r, dtype=f), torch.tensor(self.s_, dtype=f), torch.tensor(self.dw, dtype=f),
                torch.tensor(self.done, dtype=f))


class RolloutBuffer:
    """Device-resident [T, N] rollout storage (HBM, f32 / u8)."""

    def __init__(self, T: int, N: int, device, obs_dim: int = 18, act_dim: int = 3):
        self.T, self.N = int(T), int(N)
        kw = dict(device=device)
        self.obs = torch.zeros((T + 1, N, obs_dim), dtype=torch.float32, **kw)
        self.act = torch.zeros((T, N, act_dim), dtype=torch.float32, **kw)
        self.logp = torch.zeros((T, N, act_dim), dtype=torch.float32, **kw)
        self.rew = torch.zeros((T, N), dtype=torch.float32, **kw)
        self.done = torch.zeros((T, N), dtype=torch.uint8, **kw)
        self.values = torch.zeros((T + 1, N), dtype=torch.float32, **kw)
        self.adv = torch.zeros((T, N), dtype=torch.float32, **kw)
        self.vtarget = torch.zeros((T, N), dtype=torch.float32, **kw)
        self.packed = torch.zeros((T * N, 32), dtype=torch.float32, **kw)

    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in (self.obs, self.act, self.logp, self.rew, self.done,
                                                          self.values, self.adv, self.vtarget, self.packed))

    def pack(self, adv_norm):
        """Gather-friendly [T*N, 32] rows: s(18) a(3) logp(3) adv(1) v_target(1)."""
        B = self.T * self.N
        p = self.packed
        p[:, 0:18] = self.obs[:self.T].reshape(B, -1)
        p[:, 18:21] = self.act.reshape(B, -1)
        p[:, 21:24] = self.logp.reshape(B, -1)
        p[:, 24] = adv_norm.reshape(B)
        p[:, 25] = self.vtarget.reshape(B)
        return p
