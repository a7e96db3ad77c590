"""madrona_basketball_amd -- MI355X-native batched 2D basketball simulator.

Drop-in for the step path of davidj24/madrona_basketball: the module surface of
`madrona_basketball` (src/bindings.cpp:14-101) backed by one fused gfx950 HIP
step kernel (csrc/bb_kernels.hip) and a host executor for ExecMode.CPU.
"""
from . import madrona
from .madrona import ExecMode
from .simulator import SimpleGridworldSimulator, Tensor
from .recorder import TrajectoryRecorder
from ._lib import ABI_SYMBOLS, EXPORT_IDS

__all__ = ["SimpleGridworldSimulator", "Tensor", "TrajectoryRecorder", "ExecMode", "madrona", "ABI_SYMBOLS",
           "EXPORT_IDS"]
