"""Flag 2 (environment.py:257-315) against the
reference's recorded steps (tests/golden/flag2.npz, capture_flag2.py):
CPU parts -- the oracle and the host build step the state like the
reference, bit for bit; the Flag-2 orbit inputs and the env's
ellipse-fitting trainer (network_method_train, torch CPU) reproduce the
reference exactly.  The GPU drop-in (grid + fit kernels) is in
test_flag2_gpu.py."""
import numpy as np
import pytest
import torch

from conftest import R_CW, STATE_KEYS, V_CW, golden


def _state(d, prefix, j):
    return {k: d[prefix + k][j] for k in STATE_KEYS}


def test_flag2_oracle_steps_bitexact(oracle):
    """Every recorded Flag-2 step from its recorded start state: obs, state
    after, done exact; reward 0 (no danger-zone update, gating of Flag 0)."""
    d = golden("flag2")
    for j in range(len(d["r"])):
        e = oracle.OracleEnv(0.0, 6 if d["run"][j] == 0 else 50)
        e.set_state(_state(d, "b_", j))
        obs, r, done = e.step(d["pa"][j], d["ea"][j], int(d["count"][j]))
        assert np.array_equal(obs, d["obs"][j]), j
        assert r == 0.0 and d["r"][j] == 0.0 and d["r_is_int"][j] == 1
        assert done == bool(d["done"][j]), j
        st = e.get_state()
        for k in STATE_KEYS:
            assert np.array_equal(np.asarray(st[k]), np.asarray(d["a_" + k][j])), (j, k)


def test_flag2_host_build_steps_bitexact():
    """The product's host build (satenv_cpu) on all recorded steps at once."""
    from test_host_build import _planes
    from satrl.env import VecSatellites
    d = golden("flag2")
    n = len(d["r"])
    for run, max_ep in ((0, 6), (1, 50)):
        idx = np.nonzero(d["run"] == run)[0]
        env = VecSatellites(len(idx), device="cpu", d_capture=0.0, max_episode_steps=max_ep, Flag=2)
        env.set_state(*_planes(d, "b_", idx))
        obs64 = torch.empty((len(idx), 18), dtype=torch.float64)
        _, r, done = env.step(torch.tensor(d["pa"][idx]), torch.tensor(d["ea"][idx]),
                              torch.tensor(d["count"][idx], dtype=torch.int32), obs64_out=obs64)
        assert env.check_errors() == 0
        assert np.array_equal(obs64.numpy(), d["obs"][idx])
        assert np.array_equal(done.numpy(), d["done"][idx]) and not r.numpy().any()
        fa, ia = env.get_state()
        fr, ir = _planes(d, "a_", idx)
        assert torch.equal(fa, fr) and torch.equal(ia, ir)
    assert n == 12


def test_flag2_orbit_inputs_exact():
    """numerical_method_process's Incoming_parameters inputs (a, e, f,
    delta_max and its numpy type) from the recorded post-step states by the
    host restatement of real_time_data_process.calculate_orbital_elements."""
    from satrl.surrogate import rtp_orbital_elements
    d = golden("flag2")
    for j in range(len(d["r"])):
        R0 = R_CW + d["a_Pp"][j]
        V0 = V_CW + d["a_Pv"][j]
        el = rtp_orbital_elements(3.986e14, R0, V0)
        a, e, f, dm, f32 = d["orbit"][j]
        assert (el[0], el[1], el[5]) == (a, e, f), j
        assert dm == d["a_fuel_c"][j] and bool(f32) == (d["a_fuel_c_mode"][j] == 2)


def test_flag2_trainer_is_the_reference():
    """network_method_train (real_time_data_process.py:127-183) on the CPU:
    ImprovedNN's init after torch.manual_seed(seed) and every parameter after
    each recorded train step -- dropout masks included -- equal the
    reference's bit for bit, as does the loss."""
    from satrl.env import _typed
    from satrl.surrogate import network_method_train
    d = golden("flag2")
    for run in (0, 1):
        torch.manual_seed(run)
        tr = network_method_train()
        flat = lambda: torch.cat([p.detach().reshape(-1) for p in tr.net.parameters()]).numpy()
        assert np.array_equal(flat(), d[f"params0_{run}"])
        for j in np.nonzero(d["run"] == run)[0]:
            fuel = _typed(d["a_fuel_c"][j], d["a_fuel_c_mode"][j])
            tr.train(R_CW + d["a_Pp"][j], V_CW + d["a_Pv"][j], fuel, d["ell"][j])
            assert tr.all_loss[-1].item() == d["loss"][j], j
            assert np.array_equal(flat(), d["params"][j]), j


def test_flag2_reset_and_bad_flag():
    from satrl.env import VecSatellites
    env = VecSatellites(3, device="cpu", Flag=2)
    obs = env.reset(2)
    assert obs.shape == (3, 18)
    from satrl import _lib
    with pytest.raises(_lib.NativeError):
        env.reset(3)
