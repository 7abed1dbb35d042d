"""Module-name shim for ``from ppo_continuous import PPO_continuous``
(CPPO_main.py:6): satrl.ppo mirrors ppo_continuous.py:10-265."""
from satrl.ppo import Actor_Gaussian, Critic, PPO_continuous, orthogonal_init  # noqa: F401
