"""Module-name shim: ``from environment import satellites`` (CPPO_main.py:7)
resolves to the MI355X engine when this directory is on sys.path ahead of
the reference.  The class is satrl.env.satellites (environment.py:26-255)."""
from satrl.env import Box, Discrete, VecSatellites, satellites  # noqa: F401
