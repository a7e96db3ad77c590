"""One summary line of a bench.py JSON output (tools/ab_bench.sh)."""
import json
import sys

v, mode, f = sys.argv[1:]
d = [json.loads(line) for line in open(f) if line.startswith("{")][-1]
r = d["roofline"]
print(f"{v:10s} {mode:40s} {d['value'] / 1e9:7.3f} G/s  {r['kernel']:18s} {r['kernel_avg_us']:9.2f} us  "
      f"step {d['ms_per_step'] * 1e3:7.2f} us  frac {r['frac']:.3f}")
