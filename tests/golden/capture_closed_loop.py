#!/usr/bin/env python3
"""Capture the reference's UNFORCED closed-loop episodes in a fresh process
(build container ONLY; the reference never travels).

CPPO_main.test_network (CPPO_main.py:233-282) exactly as SURVEY.md §3.2 ran
it: torch.manual_seed(0), np.random.seed(0), the one_layer pursuer
checkpoint, the __main__ env constructor, d_capture 20000, max_episode_steps
64 and 1000 -- nothing else imported or run before it in the process (the
per-step trajectories of test_network.npz were recorded after other
captures in one process, and their agent forwards differ from a clean run's
by ~1e-6).  Records the per-step rewards / dones and the printed return:

  closed_loop.npz   r_64, done_64, return_64, r_1000, done_1000, return_1000

Run:  python tests/golden/capture_closed_loop.py
"""
import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from capture_golden import REF, _setup  # noqa: E402


def main():
    _setup()
    import torch
    import CPPO_main
    import environment
    out = {}
    for max_ep in (64, 1000):
        torch.manual_seed(0)
        np.random.seed(0)
        a2 = CPPO_main.args_param(max_episode_steps=max_ep, batch_size=64, max_train_steps=5000, K_epochs=3,
                                  chkpt_dir=os.path.join(REF, "model_file", "one_layer"))
        env = environment.satellites(Pursuer_position=np.array([2000000, 2000000, 1000000]),
                                     Pursuer_vector=np.array([1710, 1140, 1300]),
                                     Escaper_position=np.array([1850000, 2000000, 1000000]),
                                     Escaper_vector=np.array([1710, 1140, 1300]), d_capture=50000, args=a2)
        log = {"r": [], "done": []}
        orig_step = environment.satellites.step

        def step(self, pa, ea, c, _orig=orig_step):
            s_, r, d = _orig(self, pa, ea, c)
            log["r"].append(float(r))
            log["done"].append(int(d))
            return s_, r, d

        environment.satellites.step = step
        with contextlib.redirect_stdout(io.StringIO()) as buf:
            CPPO_main.test_network(a2, env, show_pictures=False, d_capture=20000)
        environment.satellites.step = orig_step
        printed = buf.getvalue().strip().splitlines()[-1]
        ret = 0
        for r in log["r"]:
            ret += r
        print("test_network", max_ep, "return", repr(ret), "| printed:", printed)
        out[f"r_{max_ep}"] = np.asarray(log["r"])
        out[f"done_{max_ep}"] = np.asarray(log["done"], np.uint8)
        out[f"return_{max_ep}"] = np.array(float(ret))
    np.savez_compressed(os.path.join(HERE, "closed_loop.npz"), **out)


if __name__ == "__main__":
    main()
