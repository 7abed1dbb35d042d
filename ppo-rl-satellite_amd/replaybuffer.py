"""Module-name shim for ``from replaybuffer import ReplayBuffer``
(CPPO_main.py:5): satrl.buffer.ReplayBuffer mirrors replaybuffer.py:3-38."""
from satrl.buffer import ReplayBuffer  # noqa: F401
