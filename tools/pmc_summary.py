"""Per-kernel medians of every counter under a tools/pmc_bench.sh output dir.

python tools/pmc_summary.py gpurun_out/<tag>  -> one line per (kernel, counter)
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main(d):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "bb::" not in k:
                continue
            vals[(k.split("(")[0].replace("void ", ""), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(vals.items()):
        print(f"{k:28s} {c:22s} {statistics.median(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
