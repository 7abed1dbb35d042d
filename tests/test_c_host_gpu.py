"""The C ABI from a host with no Python and no torch in its process
(examples/c_host_step, built by __graft_entry__.build()): its env rollout and
PPO minibatch step, run again on the same inputs through the Python package,
give the same results.

  * env: 2048 envs x 40 autoreset steps (episodes end at step 12 and reset
    in-kernel): obs, rewards and done flags bit for bit;
  * PPO (H 256, both nets) at mb 4096 (the bench's minibatch, 32-row
    rowpass blocks) and mb 512 (configs[3]'s per-rank minibatch, 16-row
    blocks): the f32 rowpass's H1 / dZ2, and the gradient, parameters, Adam
    moments, step counters and fc2.weight^T after the product step (k-packed
    planes, split-bf16 dW2, reduce, Adam: every kernel hand-written, no
    library tiles) bit for bit."""
import os
import subprocess

import numpy as np
import pytest
import torch


pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "c_host_step")


def _load(d, name, dtype, shape):
    return np.fromfile(os.path.join(d, name), dtype=dtype).reshape(shape)


def test_c_host_matches_the_python_path(tmp_path):
    if not os.path.exists(EXE):
        pytest.fail("examples/c_host_step is not built: run __graft_entry__.build()")
    r = subprocess.run([EXE, str(tmp_path)], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    print(r.stdout.strip())
    d = str(tmp_path)

    # ---- env ----------------------------------------------------------------------
    from satrl.env import VecSatellites
    N, T = 2048, 40
    pa = _load(d, "env_pa.f32", np.float32, (T, N, 3))
    ea = _load(d, "env_ea.f32", np.float32, (T, N, 3))
    env = VecSatellites(N, d_capture=15000.0, max_episode_steps=12)
    env.reset(0)
    rew, done = [], []
    for t in range(T):
        obs, rw, dn = env.step_autoreset(torch.tensor(pa[t], device="cuda"), torch.tensor(ea[t], device="cuda"))
        rew.append(rw.cpu().numpy())
        done.append(dn.cpu().numpy())
    assert np.array_equal(obs.cpu().numpy(), _load(d, "env_obs.f32", np.float32, (N, 18)))
    assert np.array_equal(np.stack(rew), _load(d, "env_rew.f32", np.float32, (T, N)))
    assert np.array_equal(np.stack(done), _load(d, "env_done.u8", np.uint8, (T, N)))
    assert np.stack(done).any()
    st_c = _load(d, "env_stats.f64", np.float64, (4,))
    st_py = env.stats.cpu().numpy()
    assert st_c[0] == st_py[0] and st_c[3] == st_py[3]                    # episodes, captures: exact
    assert np.allclose(st_c[1:3], st_py[1:3], rtol=1e-12)                 # sums (atomic order)

    # ---- PPO minibatch steps -----------------------------------------------------------
    for mb in (4096, 512):
        _check_ppo_step(d, mb)


def _check_ppo_step(d, mb):
    from satrl.ppo import PPOLearner
    from satrl.trainer import args_param
    H, tag = 256, f"ppo{mb}_"
    args = args_param(hidden_width=H, mini_batch_size=mb, batch_size=mb, chkpt_dir="/tmp")
    L = PPOLearner(args, "pursuer", use_graph=False)
    total = L.P.numel()
    bct_c = np.fromfile(os.path.join(d, tag + "bct.f64"), dtype=np.float64)
    assert np.array_equal(L.bct.cpu().numpy().reshape(-1), bct_c)         # same Adam bias-correction table
    assert L.lr.cpu().tolist() == [np.float32(2e-4)] * 2
    assert (L.epsilon, L.entropy_coef, L.max_action, L.adam_eps) == (0.1, 0.01, 1.6, 1e-5)
    with torch.no_grad():
        L.P.copy_(torch.from_numpy(_load(d, tag + "P0.f32", np.float32, (total,))))
        L.sync_w2t()
        for b in (L.M, L.V, L.G, L.steps):
            b.zero_()
    src = torch.from_numpy(_load(d, tag + "src.f32", np.float32, (mb, 32))).cuda()
    st = L.stepper(mb)
    H1, dZ2 = st.rowpass(src, None)
    torch.cuda.synchronize()
    assert np.array_equal(H1.cpu().numpy(), _load(d, tag + "H1.f32", np.float32, (2 * mb * H,)))
    assert np.array_equal(dZ2.cpu().numpy(), _load(d, tag + "dZ2.f32", np.float32, (2 * mb * H,)))
    st.step(src, None)
    torch.cuda.synchronize()
    out = {k: getattr(L, k).cpu().numpy() for k in ("G", "P", "M", "V", "W2T")}
    ref = {k: _load(d, f"{tag}{k}.f32", np.float32, out[k].shape) for k in out}
    assert np.array_equal(L.steps.cpu().numpy(), _load(d, tag + "steps.f64", np.float64, (2,)))
    assert st.kx(mb)                             # both hosts: the k-packed split-bf16 dW2
    for k in out:
        assert np.array_equal(out[k], ref[k]), (mb, k)
