"""Static VALU/SALU instruction count per system (tools/probe/sys_cost.hip).

python tools/sys_cost.py [--agents 2]
"""
import argparse
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=2)
    a = ap.parse_args()
    src = os.path.join(ROOT, "tools", "probe", "sys_cost.hip")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                        "-fhip-fp32-correctly-rounded-divide-sqrt", f"-DBB_N={a.agents}", "--cuda-device-only",
                        "-S", src, "-o", out], check=True)
        asm = open(out).read()
    counts = {}
    for m in re.finditer(r"^_ZN2bb(\d+)k_(\w+?)ENS_6ParamsE:(.*?)s_endpgm", asm, re.S | re.M):
        body = m.group(3)
        name = m.group(2)
        counts[name] = (len(re.findall(r"^\s+v_", body, re.M)), len(re.findall(r"^\s+s_", body, re.M)),
                        len(re.findall(r"^\s+v_\w+_f64", body, re.M)))
    base = counts.get("none", (0, 0, 0))
    print(f"{'system':20s} {'VALU':>6s} {'SALU':>6s} {'f64':>5s}   (minus load + tick + actionMask + store)")
    for k, (v, s_, f) in counts.items():
        print(f"{k:20s} {v - base[0]:6d} {s_ - base[1]:6d} {f:5d}")


if __name__ == "__main__":
    main()
