"""Build libmadrona_basketball_amd.so in-tree with hipcc for gfx950.

python -m madrona_basketball_amd.build   (or __graft_entry__.build())
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_NAME = "libmadrona_basketball_amd.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
AGENT_COUNTS = [2, 4, 6, 8, 10]
# (source, extra flags, object name): the step kernel once per agent count,
# compiled in parallel
UNITS = ([("bb_kernels.hip", [f"-DBB_N={n}"], f"bb_kernels_n{n}.o") for n in AGENT_COUNTS]
         + [("bb_common.hip", [], "bb_common.o"), ("bb_host.hip", [], "bb_host.o")])
SOURCES = sorted({u[0] for u in UNITS})
HEADERS = ["bb_math.h", "bb_rng.h", "bb_sim.h", "bb_launch.h"]
ARCH = os.environ.get("BB_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: every float op rounds on its own (bit parity host <-> gfx950)
# correctly rounded f32 divide/sqrt on the device (HIP default, made explicit)
FLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-ffp-contract=off", "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build madrona_basketball_amd)")


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "madrona_basketball_amd.h"))
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB_PATH
    cc = hipcc()
    objs = []
    build_dir = os.path.join(HERE, "_build")
    os.makedirs(build_dir, exist_ok=True)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(UNITS), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    cmds = []
    for src, extra, objname in UNITS:
        obj = os.path.join(build_dir, objname)
        cmds.append([cc, *FLAGS, *extra, "-c", os.path.join(CSRC, src), "-o", obj])
        objs.append(obj)
        if verbose:
            print(" ".join(cmds[-1]), file=sys.stderr)
    with ThreadPoolExecutor(jobs) as ex:
        for r in ex.map(lambda c: subprocess.run(c), cmds):
            r.check_returncode()
    tmp = LIB_PATH + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
