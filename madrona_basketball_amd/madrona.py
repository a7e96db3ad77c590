"""`madrona_basketball.madrona` submodule: ExecMode (scripts/env.py:31-32)."""
import enum


class ExecMode(enum.IntEnum):
    CPU = 0
    CUDA = 1  # the HIP / gfx950 executor, named as in the reference
