#!/bin/bash
# Round 4, session y: floors of the C4 shard (32 768 x 2) and C2 (8 192 x 2)
# on the final build: product, memory phases only, no systems, stream probes,
# and the per-wave phase trace.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/y
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for W in 32768 8192 65536; do
timeout -k 10 300 python3 tools/ablate.py --worlds $W --agents 2 --iters 200 --rounds 3 > $OUT/ablate_W$W.log 2>&1 || exit 1
grep -v "^trace\|^{\|amdgpu.ids" $OUT/ablate_W$W.log | sed "s|^|W=$W |"
done
