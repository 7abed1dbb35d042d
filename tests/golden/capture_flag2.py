#!/usr/bin/env python3
"""Capture golden vectors for Flag 2 (build container ONLY; reads
/root/reference read-only, through capture_golden's gym stub).

environment.satellites.step with Flag == 2 (environment.py:257-315): the
state update without a danger-zone update, reward 0, then
numerical_method_process (real_time_data_process.py:107-110 ->
RD_single_pulse.Incoming_parameters / Reachable_Domain / curve_fitting) for
env.ellipse_params and one network_method_train.train step (:146-183) of
the env's ImprovedNN.  The trainer saves MLPNet2.pth to the author's
absolute path at its 10th step (which raises here), so each run stays below
10 steps.

Fixture flag2.npz (run k = 0, 1; step j):
  pa, ea [S][3] f32, count [S], run [S], obs [S][18], r [S], r_is_int [S],
  done [S], b_*/a_* state before/after (capture_golden.STATE_KEYS),
  ell [S][2][5] env.ellipse_params, orbit [S][5] (a, e, f, delta_max,
  delta_max is np.float32) handed to Incoming_parameters, loss [S],
  params0_<k> (the trainer's initial flat parameters of run k),
  params [S][P] (the trainer's flat parameters after the step)

Run:  python tests/golden/capture_flag2.py      (~30 s)
"""
import contextlib
import io
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import capture_golden as CG  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def flat(net):
    import torch
    return torch.cat([p.detach().reshape(-1) for p in net.parameters()]).numpy().copy()


def main():
    CG._setup()
    import torch
    import CPPO_main
    import environment
    from single_pluse_model import RD_single_pulse as RD
    from single_pluse_model import real_time_data_process as RTP

    orbit_log = []
    orig_ip = RD.Incoming_parameters

    def ip(data, delta_max):
        orbit_log.append([float(data[0]), float(data[1]), float(data[5]), float(delta_max),
                          float(isinstance(delta_max, np.float32))])
        return orig_ip(data, delta_max)

    RD.Incoming_parameters = ip
    RTP.RD_single_pulse.Incoming_parameters = ip

    recs = {k: [] for k in ["pa", "ea", "count", "run", "obs", "r", "r_is_int", "done", "ell", "orbit", "loss",
                            "params"] + ["b_" + k for k in CG.STATE_KEYS] + ["a_" + k for k in CG.STATE_KEYS]}
    extra = {}
    runs = [  # (seed, steps, max_episode_steps, start state or None)
        (0, 8, 6, None),
        (1, 4, 50, dict(Pp=[40000.0, 2500.0, -800.0], Pv=[-3.5, 1.25, 0.5], Ep=[18000.0, 0.0, 0.0],
                        Ev=[0.5, -0.25, 0.0], fuel_c=300.0, fuel_t=310.0, dis=22000.0, dz=1, fuel_c_mode=3,
                        fuel_t_mode=2, vel_int=0, flag=2)),
    ]
    for k, (seed, steps, max_ep, start) in enumerate(runs):
        torch.manual_seed(seed)
        np.random.seed(seed)
        args = CPPO_main.args_param(chkpt_dir=os.path.join(CG.REF, "model_file", "one_layer"),
                                    max_episode_steps=max_ep)
        env = environment.satellites(args=args)
        env.d_capture = 0                        # train_elliptical_network(d_capture=0), CPPO_main.py:288
        extra[f"params0_{k}"] = flat(env.trian_elliptical_fitting.net)
        rng = np.random.default_rng(100 + seed)
        s = env.reset(2)
        if start is not None:
            CG.set_env_state(env, start)
        count = 0
        for t in range(steps):
            count += 1
            pa = rng.uniform(-2.0, 2.0, 3).astype(np.float32)
            ea = rng.uniform(-2.0, 2.0, 3).astype(np.float32)
            st = CG.env_state(env)
            n_orb = len(orbit_log)
            with contextlib.redirect_stdout(io.StringIO()):
                s_, r, done = env.step(pa, ea, count)
            assert len(orbit_log) == n_orb + 1
            st2 = CG.env_state(env)
            tr = env.trian_elliptical_fitting
            recs["pa"].append(pa); recs["ea"].append(ea); recs["count"].append(count); recs["run"].append(k)
            recs["obs"].append(np.asarray(s_, np.float64)); recs["r"].append(float(r))
            recs["r_is_int"].append(int(type(r) is int)); recs["done"].append(int(done))
            recs["ell"].append(np.asarray(env.ellipse_params, np.float64).reshape(2, 5))
            recs["orbit"].append(orbit_log[-1]); recs["loss"].append(float(tr.all_loss[-1].item()))
            recs["params"].append(flat(tr.net))
            for key in CG.STATE_KEYS:
                recs["b_" + key].append(st[key]); recs["a_" + key].append(st2[key])
            s = s_
            if done:
                s = env.reset(2)
                count = 0
    out = {key: np.asarray(v) for key, v in recs.items()}
    out.update(extra)
    np.savez_compressed(os.path.join(OUT, "flag2.npz"), **out)
    print("flag2.npz:", len(out["r"]), "steps; done", out["done"].tolist(), "ell finite",
          bool(np.isfinite(out["ell"]).all()))


if __name__ == "__main__":
    main()
