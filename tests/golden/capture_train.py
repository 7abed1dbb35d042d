#!/usr/bin/env python3
"""Capture the reference's training loop (build container ONLY).

CPPO_main.train_pursuer_network (CPPO_main.py:94-161) as the reference's
__main__ runs it for Sign == 0 (CPPO_main.py:326-340: max_episode_steps 64,
batch_size 64, K_epochs 3, pre_train from the one_layer checkpoint,
d_capture 15000), torch/np seed 0, for 3 episodes.  The batch fills every 64
steps, so PPO_continuous.update runs inside the loop and its minibatch
permutations come from the same global torch generator as every
choose_action draw.  Recorded per step: the pursuer's observation, both
agents' actor means and sampled actions, the pursuer's log-probs, reward and
done; after every update: the pursuer's actor/critic parameters.  Written to
train_loop.npz next to this script.  The checkpoint is copied to a scratch
directory first (save_checkpoint writes there; the reference stays
read-only).

Run:  python tests/golden/capture_train.py
"""
import contextlib
import io
import os
import shutil
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import capture_golden as cg  # noqa: E402

EPISODES = 3


def main():
    cg._setup()
    import torch
    torch.set_num_threads(1)
    import CPPO_main
    import environment
    import ppo_continuous

    ck = tempfile.mkdtemp(prefix="one_layer_")
    for f in ("agent_pursuer_actor_Gaussian", "agent_pursuer_critic"):
        shutil.copy(os.path.join(cg.REF, "model_file", "one_layer", f), ck)

    log = {"obs_in": [], "pa": [], "pmean": [], "plogp": [], "ea": [], "emean": [], "r": [], "done": [],
           "update_step": []}
    params = []
    P = ppo_continuous.PPO_continuous
    orig_init, orig_choose, orig_update = P.__init__, P.choose_action, P.update
    orig_step = environment.satellites.step

    def init(self, args_, idx):
        orig_init(self, args_, idx)
        self._cap_name = idx

    def choose(self, s):
        with torch.no_grad():
            m = self.actor(torch.unsqueeze(torch.tensor(s, dtype=torch.float), 0)).numpy().ravel()
        a, lp = orig_choose(self, s)
        if self._cap_name == "pursuer":
            log["obs_in"].append(np.asarray(s, np.float64))
            log["pa"].append(a)
            log["pmean"].append(m)
            log["plogp"].append(lp)
        else:
            log["ea"].append(a)
            log["emean"].append(m)
        return a, lp

    def update(self, rb, total_steps):
        orig_update(self, rb, total_steps)
        log["update_step"].append(len(log["r"]))
        sd = {}
        for net in ("actor", "critic"):
            for k, v in getattr(self, net).state_dict().items():
                sd[f"{net}.{k}"] = v.detach().numpy().copy()
        params.append(sd)

    def step(self, pa, ea, c):
        s_, r, d = orig_step(self, pa, ea, c)
        log["r"].append(float(r))
        log["done"].append(int(d))
        return s_, r, d

    P.__init__, P.choose_action, P.update = init, choose, update
    environment.satellites.step = step
    torch.manual_seed(0)
    np.random.seed(0)
    args = CPPO_main.args_param(max_episode_steps=64, batch_size=64, max_train_steps=EPISODES, K_epochs=3,
                                chkpt_dir=ck)
    env = environment.satellites(Pursuer_position=np.array([2000000, 2000000, 1000000]),
                                 Pursuer_vector=np.array([1710, 1140, 1300]),
                                 Escaper_position=np.array([1850000, 2000000, 1000000]),
                                 Escaper_vector=np.array([1710, 1140, 1300]), d_capture=50000, args=args)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        CPPO_main.train_pursuer_network(args, env, show_picture=False, pre_train=True, d_capture=15000)
    out = {k: np.asarray(v) for k, v in log.items()}
    for i, sd in enumerate(params):
        for k, v in sd.items():
            out[f"after{i}.{k}"] = v
    out["n_updates"] = np.array(len(params))
    path = os.path.join(cg.OUT, "train_loop.npz")
    np.savez_compressed(path, **out)
    print("steps", len(log["r"]), "updates at", log["update_step"], "dones", int(np.sum(log["done"])), "->", path)


if __name__ == "__main__":
    main()
