#!/bin/bash
# PPO fused-rollout A/B: the product build against a variant build
# (build.py --variant <name>), interleaved pairs of tools/ppo_k_sweep.py.
# Usage: bash tools/ab_ppo.sh <tag> <variant> [pairs] [worlds]
set -u
TAG=$1; V=$2; PAIRS=${3:-3}; W=${4:-8192}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
LIB=$R/madrona_basketball_amd/_variants/$V/libmadrona_basketball_amd.so
for i in $(seq "$PAIRS"); do
    for v in base "$V"; do
        if [ "$v" = base ]; then lib=""; else lib=$LIB; fi
        echo "=== pair $i $v"
        MADRONA_BB_LIB=$lib timeout -k 10 240 python3 "$R/tools/ppo_k_sweep.py" --worlds "$W" --ks "${KS:-8,32,64}" --calls 30 \
            > "$OUT/tmp.log" 2>&1 || { cat "$OUT/tmp.log"; exit 1; }
        grep -v amdgpu.ids "$OUT/tmp.log" | sed "s/^/$v: /" | tee -a "$OUT/ab.txt"
    done
done
