"""Per-kernel register / scratch / LDS usage of the built gfx950 code objects.

Reads the clang offload bundles in madrona_basketball_amd/_build/*.o and prints
llvm-readelf's AMDGPU metadata for kernels matching a pattern:
    python tools/kernel_resources.py [regex] [build dir, default madrona_basketball_amd/_build]
"""
import glob
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path):
    data = open(path, "rb").read()
    pos = 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple:
                yield data[i + off:i + off + size]
        pos = i + len(MAGIC)


def main():
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    keys = ("group_segment_fixed_size", "private_segment_fixed_size", "vgpr_count", "agpr_count",
            "vgpr_spill_count", "sgpr_spill_count")
    bdir = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "madrona_basketball_amd", "_build")
    for o in sorted(glob.glob(os.path.join(bdir, "*.o"))):
        for co in code_objects(o):
            with tempfile.NamedTemporaryFile(suffix=".co") as f:
                f.write(co)
                f.flush()
                out = subprocess.run([readelf, "--notes", f.name], capture_output=True, text=True).stdout
            cur = {}
            for line in out.splitlines():
                s = line.strip()
                if s.startswith("- .agpr_count") or s.startswith(".agpr_count"):
                    cur = {}
                m = re.match(r"-?\s*\.(\w+):\s+(.*)", s)
                if not m:
                    continue
                k, v = m.group(1), m.group(2)
                cur[k] = v
                if k == "vgpr_spill_count" and ".name" in cur or k == "wavefront_size":
                    pass
                if k == "wavefront_size":
                    name = cur.get("name", "?")
                    if pat.search(name):
                        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
                        print(f"{dem[:70]:70s} " + " ".join(f"{kk.split('_')[0]}{'/' + kk.split('_')[1] if kk.startswith(('vgpr_s', 'sgpr_s', 'group', 'private')) else ''}={cur.get(kk, '?')}" for kk in keys))
                    cur = {}


if __name__ == "__main__":
    main()
