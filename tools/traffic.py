"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into HBM
bytes per k_step launch -> profiles/traffic.json (read by bench.py).

Corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane
streaming stores.  Infinity-Cache hits are counted (not excluded).

python tools/traffic.py <fetch_dir> <write_dir> <workload_key> [--out profiles/traffic.json]
python tools/traffic.py <fetch_dir> <write_dir> W65536_PPO_R32 --ppo-fused 32
    (the fused PPO kernels: k_rollout_ppo / k_rollout_policy launches of 32
    steps, their counters per step)
python tools/traffic.py <fetch_dir> <write_dir> W65536_PPO_R32 --ppo 1
    (PPO rollout: every k_policy, k_step and k_step_ppo launch summed, per
    step = per step launch x the parts a step is split into -- 2 for the
    two-stream split; the fused rollout: --ppo 1 --ppo-k 32, a
    k_rollout_policy launch counting 32 steps)
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_launch(d, counter, kernel_sub):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kernel_sub in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel_sub} under {d}")
    return statistics.median(vals), len(vals)


def ppo_per_step(d, counter, parts, k_steps=1):
    """Sum of counter over every k_policy / k_step / k_step_ppo /
    k_rollout_policy launch, per PPO step (a k_rollout_policy launch is
    k_steps steps)."""
    tot, steps, pol = 0.0, 0, 0.0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            if "k_step<" in k or "k_step_ppo<" in k:
                tot += float(r["Counter_Value"])
                steps += 1
            elif "k_rollout_policy<" in k:
                tot += float(r["Counter_Value"])
                steps += k_steps
            elif "k_policy" in k:
                tot += float(r["Counter_Value"])
                pol += float(r["Counter_Value"])
    if not steps:
        raise SystemExit(f"no k_step {counter} rows under {d}")
    n = steps / parts
    return tot / n, pol / n, steps


def fused_per_step(d, counter, k_steps):
    """A fused PPO rollout (k_rollout_ppo / k_rollout_policy: k_steps steps per
    launch; the warm-up's plain k_step launches are not PPO steps): the
    counter summed over those launches, per step."""
    tot, launches = 0.0, 0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and ("k_rollout_ppo<" in r["Kernel_Name"]
                                                 or "k_rollout_policy<" in r["Kernel_Name"]):
                tot += float(r["Counter_Value"])
                launches += 1
    if not launches:
        raise SystemExit(f"no fused PPO {counter} rows under {d}")
    return tot / (launches * k_steps), launches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("key")
    ap.add_argument("--kernel", default="k_step<2, 0>")
    ap.add_argument("--ppo", type=int, default=0, help="PPO rollout mode: parts per step (1 or 2)")
    ap.add_argument("--ppo-k", type=int, default=1, help="PPO rollout mode: steps per k_rollout_policy launch")
    ap.add_argument("--note", default="")
    ap.add_argument("--div", type=int, default=1, help="units (steps) per launch: the entry is per unit")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles", "traffic.json"))
    ap.add_argument("--ppo-fused", type=int, default=0, help="fused PPO rollout: steps per launch")
    a = ap.parse_args()
    try:
        data = json.load(open(a.out))
    except (OSError, ValueError):
        data = {}
    if a.ppo_fused:
        fk, nf = fused_per_step(a.fetch_dir, "FETCH_SIZE", a.ppo_fused)
        wk, nw = fused_per_step(a.write_dir, "WRITE_SIZE", a.ppo_fused)
        fetch, write = 2.0 * fk * 1024.0, wk * 1024.0
        data[a.key] = {
            "bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
            "per": f"PPO step (fused rollout launches of {a.ppo_fused} steps: their counters / steps)",
            "launches": [nf, nw], "correction": "FETCH_SIZE x2 (gfx950 half-count), KiB -> bytes",
            "source": a.note,
        }
        json.dump(data, open(a.out, "w"), indent=1, sort_keys=True)
        print(json.dumps(data[a.key]))
        return
    if a.ppo:
        fk, fpol, nf = ppo_per_step(a.fetch_dir, "FETCH_SIZE", a.ppo, a.ppo_k)
        wk, wpol, nw = ppo_per_step(a.write_dir, "WRITE_SIZE", a.ppo, a.ppo_k)
        fetch, write = 2.0 * fk * 1024.0, wk * 1024.0
        pol = 2.0 * fpol * 1024.0 + wpol * 1024.0
        data[a.key] = {
            "bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
            "k_policy_bytes": pol, "k_step_bytes": fetch + write - pol,
            "per": f"PPO step ({a.ppo} part(s): every policy / step / fused launch of the run / (steps / parts))",
            "k_step_launches": [nf, nw], "correction": "FETCH_SIZE x2 (gfx950 half-count), KiB -> bytes",
            "source": a.note,
        }
        json.dump(data, open(a.out, "w"), indent=1, sort_keys=True)
        print(json.dumps(data[a.key]))
        return
    fk, nf = per_launch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    wk, nw = per_launch(a.write_dir, "WRITE_SIZE", a.kernel)
    fetch = 2.0 * fk * 1024.0 / a.div
    write = wk * 1024.0 / a.div
    data[a.key] = {
        "bytes_per_launch": fetch + write,
        "per": "launch" if a.div == 1 else f"1/{a.div} of a launch (one step)",
        "fetch_bytes": fetch,
        "write_bytes": write,
        "raw_FETCH_SIZE_KiB": fk,
        "raw_WRITE_SIZE_KiB": wk,
        "launches": [nf, nw],
        "correction": "FETCH_SIZE x2 (gfx950 half-count), KiB -> bytes",
        "kernel": a.kernel,
        "source": a.note,
    }
    json.dump(data, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(data[a.key]))


if __name__ == "__main__":
    main()
