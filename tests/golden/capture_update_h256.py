#!/usr/bin/env python3
"""Capture seeded PPO_continuous.update() runs of the reference at the
product's hidden widths, build container ONLY.

Imports qiaobeibei/PPO-RL-Satellite from /root/reference (read-only, the
gym stub of capture_golden.py) and records ``update_h256.npz`` (H = 256,
configs[2] / configs[3]) and ``update_h64.npz`` (H = 64, configs[1]) next
to this script: data only, the reference never travels.

The minibatch shapes are the ones the product's kernels are chosen by
(satrl/ppo.py FusedMinibatch):
  kx      B 8192, mb 4096, K 2   the 32-row rowpass writing k-packed bf16
                                 planes + dw2_kx (the bench's configs[2] path)
  short   B 2048, mb  512, K 2   configs[3]'s per-rank minibatch (16-row
                                 rowpass; 4096 / 8 ranks)
  ragged  B 4873, mb 4096, K 2   one kx minibatch + a 777-row ragged tail
                                 (BatchSampler drop_last=False)
  k10     B 8192, mb 4096, K 10  the bench's epoch count: 20 Adam steps
and at H = 64 (every minibatch: the rowpass with the dW2 product fused in,
satrl_ppo_rowpass_dw2, then reduce and Adam):
  cfg1    B 8192, mb 4096, K 2   configs[1]'s minibatch (4096 envs)
  short   B 2048, mb  512, K 2
  ragged  B 4873, mb 4096, K 2
  k10     B 8192, mb 4096, K 10

Per case: the ReplayBuffer contents, the K epochs' SubsetRandomSampler
permutations (drawn from the same torch generator state update() starts
from), the parameters before and after ppo_continuous.py:191-242, and lr
after the decay.  The buffer is synthetic (reference choose_action for a
and logp on N(0, 4) states), the networks the reference's own orthogonal
init.

Run:  python tests/golden/capture_update_h256.py [256] [64]   (~1 minute each)
"""
import contextlib
import io
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from capture_golden import OUT, REF, _setup  # noqa: E402

CASES = [("kx", 8192, 4096, 2, 1001), ("short", 2048, 512, 2, 1002), ("ragged", 4873, 4096, 2, 1003),
         ("k10", 8192, 4096, 10, 1004)]
CASES_H64 = [("cfg1", 8192, 4096, 2, 2001), ("short", 2048, 512, 2, 2002), ("ragged", 4873, 4096, 2, 2003),
             ("k10", 8192, 4096, 10, 2004)]


def capture_case(name, B, mb, K, seed, CPPO_main, ppo_continuous, replaybuffer, H=256):
    import torch
    from torch.utils.data.sampler import BatchSampler, SubsetRandomSampler
    torch.manual_seed(seed)
    np.random.seed(seed)
    a = CPPO_main.args_param(batch_size=B, mini_batch_size=mb, hidden_width=H, K_epochs=K,
                             max_train_steps=5000, chkpt_dir="/nonexistent")
    a.state_dim, a.action_dim, a.max_action = 18, 3, 1.6
    with contextlib.redirect_stdout(io.StringIO()):
        agent = ppo_continuous.PPO_continuous(a, "pursuer")
    p0 = {("actor." + k): v.detach().clone().numpy() for k, v in agent.actor.state_dict().items()}
    p0.update({("critic." + k): v.detach().clone().numpy() for k, v in agent.critic.state_dict().items()})
    rng = np.random.default_rng(seed)
    # N(0, 2^2) states: fc1 in its working range.  (Rows at the raw env scale,
    # ~3e5, were tried and dropped: there fc1's pre-activation is a sum of
    # ~1e4-sized terms cancelling to O(1), so tanh' and with it dW1 depend on
    # fc1's summation order -- f64 instead of f32 sums moved the parameters by
    # 2e-4 on the CPU, 25 % of the update: a fixture no f32 engine can match.)
    S = 2.0 * rng.standard_normal((B, 18))
    S_ = S + 0.05 * rng.standard_normal((B, 18))
    R = rng.standard_normal(B) * 3.0
    DONE = (rng.random(B) < 0.01).astype(np.float64)
    DW = np.maximum(DONE, (rng.random(B) < 0.005).astype(np.float64))
    buf = replaybuffer.ReplayBuffer(a)
    for i in range(B):
        act, lp = agent.choose_action(S[i])
        buf.store(S[i], act, lp, R[i], S_[i], DW[i], DONE[i])
    # the permutations update() will draw: sample them, then rewind the generator
    st = torch.get_rng_state()
    perms = [np.concatenate([np.asarray(ix) for ix in BatchSampler(SubsetRandomSampler(range(B)), mb, False)])
             for _ in range(K)]
    torch.set_rng_state(st)
    total_steps = 123
    agent.update(buf, total_steps)
    p1 = {("actor." + k): v.detach().clone().numpy() for k, v in agent.actor.state_dict().items()}
    p1.update({("critic." + k): v.detach().clone().numpy() for k, v in agent.critic.state_dict().items()})
    # (f32: exactly what ReplayBuffer.numpy_to_tensor makes of the f64 rows)
    f32 = lambda x: np.asarray(x, np.float32)  # noqa: E731
    out = {"s": f32(buf.s), "a": f32(buf.a), "logp": f32(buf.a_logprob), "r": f32(buf.r), "s_": f32(buf.s_),
           "dw": f32(buf.dw), "done": f32(buf.done),
           "perms": np.stack(perms), "total_steps": np.array(total_steps),
           "hp": np.array([B, mb, H, K, a.max_train_steps, a.lr_a, a.lr_c, a.gamma, a.lamda, a.epsilon,
                           a.entropy_coef]),
           "lr_after": np.array([agent.optimizer_actor.param_groups[0]["lr"],
                                 agent.optimizer_critic.param_groups[0]["lr"]])}
    for k, v in p0.items():
        out["p0." + k] = v
    for k, v in p1.items():
        out["p1." + k] = v
    move = max(float(np.abs(p1[k] - p0[k]).max()) for k in p0)
    print(f"H {H} {name}: B {B} mb {mb} K {K}: max parameter movement {move:.3e}")
    return {f"{name}.{k}": v for k, v in out.items()}


def main():
    _setup()
    import torch
    torch.set_num_threads(1)
    import CPPO_main
    import ppo_continuous
    import replaybuffer
    which = sys.argv[1:] or ["256", "64"]
    for H, cases, fname in ((256, CASES, "update_h256.npz"), (64, CASES_H64, "update_h64.npz")):
        if str(H) not in which:
            continue
        fx = {}
        for case in cases:
            fx.update(capture_case(*case, CPPO_main, ppo_continuous, replaybuffer, H=H))
        np.savez_compressed(os.path.join(OUT, fname), **fx)


if __name__ == "__main__":
    main()
