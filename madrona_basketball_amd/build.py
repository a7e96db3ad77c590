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
# MachineLICM hoists the f64 polynomial constants of bb_math.h out of
# k_rollout's step loop and then spills them (628 B/lane of scratch); without
# it they are rematerialised in place.  k_step is unaffected (same VGPRs).
KERNEL_FLAGS = ["-mllvm", "-disable-machine-licm"]
# Per agent count: the max-ILP machine scheduler for the N = 2 agent-lane
# kernels (A/B, profiles/r02/t_flags_ab.txt: k_step<2> 21.7-21.8 -> 21.5 us at
# 65 536 worlds, 13.1 -> 12.8 us at 8 192; K=32 rollout 518-535 -> 485 us;
# max-memory-clause and iterative-ilp are slower, v_sched_strategy_ab.txt).
# The shared-world kernels (N >= 4) keep the default: N = 6 and 10 looked
# 1-2 % faster in one A/B (t_ilp_shared_ab.txt) but not on a second box
# (r02v: 141.1 / 310.5 us), N = 4 and 8 were slower.
MAX_ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
N_FLAGS = {2: MAX_ILP}
# (source, extra flags, object name): the step kernel once per agent count,
# compiled in parallel
UNITS = ([("bb_kernels.hip", [f"-DBB_N={n}", *KERNEL_FLAGS, *N_FLAGS.get(n, [])], f"bb_kernels_n{n}.o")
          for n in AGENT_COUNTS]
         + [("bb_common.hip", [], "bb_common.o"), ("bb_host.hip", [], "bb_host.o"),
            ("bb_policy.hip", [], "bb_policy.o")])
SOURCES = sorted({u[0] for u in UNITS})
HEADERS = ["bb_math.h", "bb_rng.h", "bb_sim.h", "bb_launch.h", "bb_policy.h"]
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


def build(force: bool = False, verbose: bool = False, variant: str | None = None,
          defines: list[str] | None = None, extra_flags: list[str] | None = None) -> str:
    """Build the library; a `variant` (diagnostics: A/B timing of compile-time
    alternatives) goes to _variants/<variant>/ with extra -D `defines` and is
    loaded only when MADRONA_BB_LIB points at it."""
    lib_path = LIB_PATH if variant is None else os.path.join(HERE, "_variants", variant, LIB_NAME)
    if variant is None and not force and not _stale():
        return LIB_PATH
    cc = hipcc()
    objs = []
    build_dir = os.path.join(HERE, "_build" if variant is None else os.path.join("_variants", variant, "_build"))
    os.makedirs(build_dir, exist_ok=True)
    from concurrent.futures import ThreadPoolExecutor
    jobs = max(1, min(len(UNITS), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    cmds = []
    for src, extra, objname in UNITS:
        obj = os.path.join(build_dir, objname)
        cmds.append([cc, *FLAGS, *extra, *[f"-D{d}" for d in (defines or [])], *(extra_flags or []), "-c",
                     os.path.join(CSRC, src), "-o", obj])
        objs.append(obj)
        if verbose:
            print(" ".join(cmds[-1]), file=sys.stderr)
    with ThreadPoolExecutor(jobs) as ex:
        for r in ex.map(lambda c: subprocess.run(c), cmds):
            r.check_returncode()
    tmp = lib_path + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib_path)
    return lib_path


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--variant", default=None, help="diagnostic build under _variants/<name>/")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra define for a variant")
    ap.add_argument("--flag", dest="flags", action="append", default=[], help="extra hipcc flag for a variant")
    a = ap.parse_args()
    print(build(force=a.force, verbose=True, variant=a.variant, defines=a.defines, extra_flags=a.flags))
