"""Replay of a captured reference PPO_continuous.update() (tests/golden/
capture_golden.py "update_case", capture_update_h256.py "update_h256")
through the drop-in PPO_continuous, on the GPU learner or the host one."""
import numpy as np
import torch

from conftest import golden


def _args(**kw):
    from satrl.trainer import args_param
    a = args_param(chkpt_dir="/tmp", **kw)
    a.state_dim, a.action_dim, a.max_action = 18, 3, 1.6
    return a


def width_case(H, name):
    """One case of update_h<H>.npz (tests/golden/capture_update_h256.py) as
    {key: array}."""
    u = golden(f"update_h{H}")
    return {k[len(name) + 1:]: u[k] for k in u.files if k.startswith(name + ".")}


def h256_case(name):
    return width_case(256, name)


def h64_case(name):
    return width_case(64, name)


def run_reference_update(u, device=None, atol=5e-5):
    """ppo_continuous.py:191-250 through the drop-in PPO_continuous on a
    captured case (the reference's buffer, minibatch permutations and
    parameters before / after): returns the worst absolute parameter diff.
    ``u`` maps the capture's keys (hp, s, a, ..., p0.*, p1.*)."""
    from satrl.buffer import ReplayBuffer
    from satrl.ppo import PPO_continuous
    B, mb, H, K, mts, lr_a, lr_c, gamma, lamda, eps, ent = u["hp"]
    args = _args(batch_size=int(B), mini_batch_size=int(mb), hidden_width=int(H), K_epochs=int(K),
                 max_train_steps=int(mts))
    agent = PPO_continuous(args, "pursuer", device=device)
    keys = list(u.keys())
    sd_a = {k[len("p0.actor."):]: torch.tensor(u[k]) for k in keys if k.startswith("p0.actor.")}
    sd_c = {k[len("p0.critic."):]: torch.tensor(u[k]) for k in keys if k.startswith("p0.critic.")}
    agent.actor.load_state_dict(sd_a)
    agent.critic.load_state_dict(sd_c)
    buf = ReplayBuffer(args)
    for i in range(int(B)):
        buf.store(u["s"][i], u["a"][i], u["logp"][i], u["r"][i], u["s_"][i], u["dw"][i], u["done"][i])
    # reproduce the reference's torch global RNG state: the fixture's perms were
    # drawn right after the buffer was filled; replay them through the sampler
    perms = u["perms"]
    import torch.utils.data.sampler as S
    orig = S.SubsetRandomSampler.__iter__
    it = iter(perms)

    def fake_iter(self):
        return iter(next(it).tolist())
    S.SubsetRandomSampler.__iter__ = fake_iter
    try:
        agent.update(buf, int(u["total_steps"]))
    finally:
        S.SubsetRandomSampler.__iter__ = orig
    worst = 0.0
    nsteps = int(K) * int(np.ceil(B / mb))
    for k in keys:
        if not k.startswith("p1."):
            continue
        name = k[3:]
        net, pname = name.split(".", 1)
        got = dict((agent.actor if net == "actor" else agent.critic).state_dict())[pname].cpu().numpy()
        ref = u[k]
        p0 = u["p0." + name]
        step_ref = np.abs(ref - p0).max()
        diff = np.abs(got - ref)
        worst = max(worst, float(diff.max()))
        assert np.allclose(got, ref, rtol=0, atol=atol), (name, diff.max(), step_ref)
    print(f"update parity (H {int(H)}, B {int(B)}, mb {int(mb)}, K {int(K)}): worst abs param diff {worst:.3e} "
          f"after {nsteps} Adam steps")
    la, lc = agent.L.lr_now
    # lr lives in an f32 device tensor (the reference keeps a python float)
    assert abs(la - u["lr_after"][0]) <= 1e-6 * u["lr_after"][0] and abs(lc - u["lr_after"][1]) <= 1e-6 * u["lr_after"][1]
    return worst
