"""The captured reference update() cases replayed through the host drop-in
(PPO_continuous(device="cpu"): torch CPU autograd, clip_grad_norm_ and Adam
in ppo_continuous.py:212-239's order, BASELINE configs[0]'s path).  This pins
the fixtures and the replay harness the GPU tests (test_ppo_gpu.py
test_update_matches_reference*) share, on any host: with one torch thread,
as the captures ran, every parameter after the update is bit for bit the
reference's."""
import pytest
import torch

from conftest import golden
from update_replay import h64_case, h256_case, run_reference_update


@pytest.fixture
def one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)          # the captures ran single-threaded: the same CPU reduction order
    yield
    torch.set_num_threads(n)


def test_host_update_matches_reference_h64(one_thread):
    u = golden("update_case")
    assert run_reference_update({k: u[k] for k in u.files}, device="cpu", atol=0.0) == 0.0


@pytest.mark.parametrize("case", ["kx", "short", "ragged", "k10"])
def test_host_update_matches_reference_h256(one_thread, case):
    assert run_reference_update(h256_case(case), device="cpu", atol=0.0) == 0.0


@pytest.mark.parametrize("case", ["cfg1", "short", "ragged", "k10"])
def test_host_update_matches_reference_h64_configs1(one_thread, case):
    """H = 64 at configs[1]'s minibatch (4096 rows), a short one and a ragged
    tail (update_h64.npz)."""
    assert run_reference_update(h64_case(case), device="cpu", atol=0.0) == 0.0
