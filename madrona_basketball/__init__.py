"""`import madrona_basketball as mba` drop-in alias (scripts/env.py:1).

Re-exports the MI355X-native implementation so the reference's scripts run
unchanged: mba.SimpleGridworldSimulator, mba.madrona.ExecMode.
"""
import sys as _sys

from madrona_basketball_amd import SimpleGridworldSimulator, Tensor, madrona  # noqa: F401

_sys.modules[__name__ + ".madrona"] = madrona
