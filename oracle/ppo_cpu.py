"""oracle/ppo_cpu.py -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

The learning side of the reference's training iteration on host cores, in
torch-CPU f32 exactly as the reference computes it, so that the CPU baseline
of bench.py is a whole PPO iteration (rollout + GAE + update) like the GPU
``value``, not only the env step:

* ``choose_action`` for a batch of states -- ppo_continuous.py:176-189
  (Actor_Gaussian ppo_continuous.py:61-101: fc1 -> tanh -> fc2 -> tanh ->
  1.6 * tanh(mean_layer), std = exp(log_std); Normal sample, clamp +-1.6,
  per-dim log_prob);
* critic values -- ppo_continuous.py:103-134, 200-201;
* one minibatch of the update -- ppo_continuous.py:213-239: clipped
  surrogate + 0.01 entropy, backward, clip_grad_norm_(0.5), Adam(eps 1e-5);
  then the critic's MSE, backward, clip, Adam.

The product never imports this module.
"""
from __future__ import annotations

import time

import torch
import torch.nn as nn
import torch.nn.functional as F


def _ortho(layer, gain=1.0):
    nn.init.orthogonal_(layer.weight, gain=gain)       # ppo_continuous.py:10-12
    nn.init.constant_(layer.bias, 0)


class _Actor(nn.Module):
    def __init__(self, H):
        super().__init__()
        self.fc1, self.fc2, self.mean_layer = nn.Linear(18, H), nn.Linear(H, H), nn.Linear(H, 3)
        self.log_std = nn.Parameter(torch.zeros(1, 3))
        _ortho(self.fc1)
        _ortho(self.fc2)
        _ortho(self.mean_layer, gain=0.01)

    def forward(self, s):
        s = torch.tanh(self.fc1(s))
        s = torch.tanh(self.fc2(s))
        return 1.6 * torch.tanh(self.mean_layer(s))


class _Critic(nn.Module):
    def __init__(self, H):
        super().__init__()
        self.fc1, self.fc2, self.fc3 = nn.Linear(18, H), nn.Linear(H, H), nn.Linear(H, 1)
        for l in (self.fc1, self.fc2, self.fc3):
            _ortho(l)

    def forward(self, s):
        return self.fc3(torch.tanh(self.fc2(torch.tanh(self.fc1(s)))))


class CpuPPO:
    def __init__(self, H=256, lr=2e-4, epsilon=0.1, entropy_coef=0.01, seed=0):
        torch.manual_seed(seed)
        self.actor, self.critic = _Actor(H), _Critic(H)
        self.opt_a = torch.optim.Adam(self.actor.parameters(), lr=lr, eps=1e-5)
        self.opt_c = torch.optim.Adam(self.critic.parameters(), lr=lr, eps=1e-5)
        self.epsilon, self.entropy_coef = epsilon, entropy_coef

    @torch.no_grad()
    def choose_action(self, s):
        mean = self.actor(s)
        dist = torch.distributions.Normal(mean, torch.exp(self.actor.log_std.expand_as(mean)))
        a = torch.clamp(dist.sample(), -1.6, 1.6)
        return a, dist.log_prob(a)

    @torch.no_grad()
    def values(self, s):
        return self.critic(s)

    def minibatch(self, s, a, lp_old, adv, vt):
        mean = self.actor(s)
        dist = torch.distributions.Normal(mean, torch.exp(self.actor.log_std.expand_as(mean)))
        ent = dist.entropy().sum(1, keepdim=True)
        ratios = torch.exp(dist.log_prob(a).sum(1, keepdim=True) - lp_old.sum(1, keepdim=True))
        surr1 = ratios * adv
        surr2 = torch.clamp(ratios, 1 - self.epsilon, 1 + self.epsilon) * adv
        actor_loss = -torch.min(surr1, surr2) - self.entropy_coef * ent
        self.opt_a.zero_grad()
        actor_loss.mean().backward()
        torch.nn.utils.clip_grad_norm_(self.actor.parameters(), 0.5)
        self.opt_a.step()
        critic_loss = F.mse_loss(vt, self.critic(s))
        self.opt_c.zero_grad()
        critic_loss.backward()
        torch.nn.utils.clip_grad_norm_(self.critic.parameters(), 0.5)
        self.opt_c.step()


def time_learning_side(n_envs, H, mb, threads, policy_steps=8, minibatches=24, seed=0):
    """Seconds per rollout step of both agents' choose_action on n_envs
    states, per critic-value pass over n_envs states, and per update
    minibatch of mb rows, on `threads` host threads (bounded samples)."""
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(seed)
    pur, eva = CpuPPO(H, seed=seed), CpuPPO(H, seed=seed + 1)
    s = torch.randn((n_envs, 18), generator=g)
    pur.choose_action(s)

    def best_of(rounds, reps, fn):
        # the fastest of `rounds` samples of `reps` calls: the host is shared
        # with other jobs, and a slow sample measures them, not this code
        best = float("inf")
        for _ in range(rounds):
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            best = min(best, (time.perf_counter() - t0) / reps)
        return best

    def both():
        pur.choose_action(s)
        eva.choose_action(s)
    t_pol = best_of(3, max(1, policy_steps // 3), both)
    t_val = best_of(2, 1, lambda: pur.values(s))
    rows = torch.randn((mb, 26), generator=g)
    sa, aa = rows[:, :18], rows[:, 18:21].clamp(-1.6, 1.6)
    lp, adv, vt = -1.0 - rows[:, 21:24].abs(), rows[:, 24:25], rows[:, 25:26]
    pur.minibatch(sa, aa, lp, adv, vt)
    t_mb = best_of(3, max(1, minibatches // 3), lambda: pur.minibatch(sa, aa, lp, adv, vt))
    return t_pol, t_val, t_mb
