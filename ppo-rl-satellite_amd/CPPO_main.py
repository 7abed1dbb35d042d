"""Module-name shim for CPPO_main.py: the config surface and training loops
(CPPO_main.py:13-282) from satrl.trainer, plus the vectorised engine.

    python CPPO_main.py [--test | --train-pursuer | --train-evader] ...

runs the reference's __main__ choices (CPPO_main.py:324-345) on the
drop-in classes; --vec runs the N-env engine instead."""
import argparse

import numpy as np

from satrl.env import satellites
from satrl.trainer import (VecTrainer, args_param, test_network, train_elliptical_network,  # noqa: F401
                           train_evader_network, train_pursuer_network)


def main():
    ap = argparse.ArgumentParser()
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--test", action="store_true", help="Sign == 1 (the reference default)")
    g.add_argument("--train-pursuer", action="store_true", help="Sign == 0, pursuer part")
    g.add_argument("--train-evader", action="store_true", help="Sign == 0, evader part")
    g.add_argument("--train-ellipse", action="store_true", help="Sign == 2: train_elliptical_network (Flag 2)")
    g.add_argument("--vec", action="store_true", help="vectorised engine iterations")
    ap.add_argument("--chkpt-dir", default="model_file/one_layer")
    ap.add_argument("--episodes", type=int, default=None)
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--iterations", type=int, default=1)
    ap.add_argument("--device", default=None,
                    help="'cpu': the drop-in on host cores (env host build + torch-CPU agents; BASELINE configs[0])")
    a = ap.parse_args()
    # CPPO_main.py:326-334
    args = args_param(max_episode_steps=64, batch_size=64, max_train_steps=5000, K_epochs=3, chkpt_dir=a.chkpt_dir,
                      device=a.device)
    if a.vec:
        args = args_param(max_episode_steps=1000, num_envs=a.num_envs, horizon=2048, batch_size=a.num_envs * 2048,
                          mini_batch_size=4096, hidden_width=256, K_epochs=10, chkpt_dir=a.chkpt_dir)
        tr = VecTrainer(args, flag=0, d_capture=15000.0)
        for _ in range(a.iterations):
            print(tr.iteration())
        return
    env = satellites(Pursuer_position=np.array([2000000, 2000000, 1000000]),
                     Pursuer_vector=np.array([1710, 1140, 1300]),
                     Escaper_position=np.array([1850000, 2000000, 1000000]),
                     Escaper_vector=np.array([1710, 1140, 1300]),
                     d_capture=50000, args=args, device=a.device)
    if a.train_pursuer:
        train_pursuer_network(args, env, show_picture=False, pre_train=True, d_capture=15000, max_episodes=a.episodes)
    elif a.train_evader:
        train_evader_network(args, env, show_picture=False, pre_train=False, d_capture=15000, max_episodes=a.episodes)
    elif a.train_ellipse:                                    # CPPO_main.py:342-343
        train_elliptical_network(args, env, epsiodes=a.episodes or 500, d_capture=0)
    else:
        test_network(args, env, show_pictures=False, d_capture=20000)


if __name__ == "__main__":
    main()
