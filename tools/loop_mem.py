"""Memory operations and vector-memory waits, in code order, of a kernel's
outermost loop (the largest backward branch) in the built gfx950 code object:
    python tools/loop_mem.py <mangled-name-regex> [object basename, default bb_kernels_n2]
A spill reload (scratch_load) or global load issued after a step's stores, and
the s_waitcnt vmcnt that retires it, wait for all of those stores."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_resources import ROOT, code_objects  # noqa: E402


def main():
    pat = re.compile(sys.argv[1])
    obj = sys.argv[2] if len(sys.argv) > 2 else "bb_kernels_n2"
    co = next(code_objects(os.path.join(ROOT, "madrona_basketball_amd", "_build", obj + ".o")))
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", f.name],
                             capture_output=True, text=True).stdout.split("\n")
    start = next(i for i, l in enumerate(dis) if re.match(r"^[0-9a-f]+ <", l) and pat.search(l))
    end = next((i for i in range(start + 1, len(dis)) if re.match(r"^[0-9a-f]+ <", dis[i])), len(dis))
    ins = []
    for l in dis[start + 1:end]:
        m = re.match(r"\s*(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", l)
        if m:
            ins.append((m.group(1), m.group(2), int(m.group(3), 16)))
    best = None
    for k, (op, arg, a) in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            try:
                imm = int(arg.split()[0])
            except ValueError:
                continue
            imm = imm - 65536 if imm >= 32768 else imm
            if imm < 0 and (best is None or -imm > best[0]):
                best = (-imm, k, a + 4 + imm * 4)
    _, kend, tgt = best
    kstart = min(k for k, (op, arg, a) in enumerate(ins) if a >= tgt)
    out, prev, cnt = [], None, 0
    for op, arg, a in ins[kstart:kend + 1]:
        if not ("store" in op or "load" in op or (op == "s_waitcnt" and "vmcnt" in arg)):
            continue
        key = op + (" " + arg.split()[0] if op == "s_waitcnt" else "")
        if key == prev:
            cnt += 1
        else:
            if prev:
                out.append(f"{prev} x{cnt}" if cnt > 1 else prev)
            prev, cnt = key, 1
    out.append(f"{prev} x{cnt}" if cnt > 1 else prev)
    print(f"loop: {kend - kstart + 1} instructions")
    print("\n".join(out))


if __name__ == "__main__":
    main()
