"""Per-phase kernel durations of a rocprofv3 --kernel-trace run of bench.py.

bench.py launches the step kernel in this order: `warmup` untimed steps, the
`steps` timed steps, a second pass of `steps` timed with HIP events (the
line's roofline.kernel_avg_us), then (unless --no-e2e) `steps` steps of the
end-to-end leg.  This splits the trace into those phases so the line's
roofline fraction can be recomputed from the committed profile.

python tools/prof_phases.py <run_kernel_trace.csv> --kernel "k_step<2, 0" --warmup 30 --steps 300
    [--bytes-per-launch 99090432] [--peak-gbs 8000]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--bytes-per-launch", type=float, default=None)
    ap.add_argument("--peak-gbs", type=float, default=8000.0)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    w, k = a.warmup, a.steps
    phases = {"warmup": (0, w), "timed": (w, w + k), "event_pass": (w + k, w + 2 * k), "e2e": (w + 2 * k, w + 3 * k)}
    out = {"kernel": a.kernel, "calls": len(us), "phases": {}}
    for name, (lo, hi) in phases.items():
        x = us[lo:hi]
        if not x:
            continue
        e = {"calls": len(x), "mean_us": statistics.mean(x), "median_us": statistics.median(x)}
        if a.bytes_per_launch:
            e["frac"] = a.bytes_per_launch / (e["mean_us"] * 1e-6) / 1e9 / a.peak_gbs
        out["phases"][name] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
