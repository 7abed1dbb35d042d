"""Plain PyTorch fp32 reference of the PPO minibatch step
(ppo_continuous.py:216-239), used only to check the fused HIP kernels."""
import copy
import math

import torch
import torch.nn.functional as F


def actor_loss(actor, s, a, lp_old, adv, epsilon, entropy_coef):
    mean = actor(s)
    std = torch.exp(actor.log_std.expand_as(mean))
    dist = torch.distributions.Normal(mean, std, validate_args=False)
    dist_entropy = dist.entropy().sum(1, keepdim=True)
    a_logprob_now = dist.log_prob(a)
    ratios = torch.exp(a_logprob_now.sum(1, keepdim=True) - lp_old.sum(1, keepdim=True))
    surr1 = ratios * adv
    surr2 = torch.clamp(ratios, 1 - epsilon, 1 + epsilon) * adv
    return (-torch.min(surr1, surr2) - entropy_coef * dist_entropy).mean()


def critic_loss(critic, s, vt):
    return F.mse_loss(vt, critic(s))


def reference_step(actor, critic, rows, epsilon=0.1, entropy_coef=0.01, lr=2e-4, eps=1e-5, clip=True):
    """One reference minibatch step on copies of the modules; returns
    (grads dict, params-after dict) keyed like PPOLearner.flat_views."""
    actor = copy.deepcopy(actor)
    critic = copy.deepcopy(critic)
    for p in list(actor.parameters()) + list(critic.parameters()):
        p.data = p.data.contiguous().clone()
        p.requires_grad_(True)
    s, a, lp, adv, vt = rows[:, 0:18], rows[:, 18:21], rows[:, 21:24], rows[:, 24:25], rows[:, 25:26]
    oa = torch.optim.Adam(actor.parameters(), lr=lr, eps=eps)
    oc = torch.optim.Adam(critic.parameters(), lr=lr, eps=eps)
    oa.zero_grad()
    actor_loss(actor, s, a, lp, adv, epsilon, entropy_coef).backward()
    grads = {"actor." + n: p.grad.detach().clone() for n, p in actor.named_parameters()}
    if clip:
        torch.nn.utils.clip_grad_norm_(actor.parameters(), 0.5)
    oa.step()
    oc.zero_grad()
    critic_loss(critic, s, vt).backward()
    grads.update({"critic." + n: p.grad.detach().clone() for n, p in critic.named_parameters()})
    if clip:
        torch.nn.utils.clip_grad_norm_(critic.parameters(), 0.5)
    oc.step()
    params = {"actor." + n: p.detach().clone() for n, p in actor.named_parameters()}
    params.update({"critic." + n: p.detach().clone() for n, p in critic.named_parameters()})
    return grads, params
