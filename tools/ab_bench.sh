#!/bin/bash
# A/B timing of diagnostic variant builds (build.py --variant NAME -D ...):
# the step bench and the rollout bench per variant ("base" = the product lib).
# Usage: [MODES='bench args|bench args'] bash tools/ab_bench.sh <tag> <variant>...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib=$ROOT/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    IFS='|' read -ra MODE_LIST <<< "${MODES:---steps 512 --warmup 64|--steps 512 --warmup 64 --rollout 32}"
    for mode in "${MODE_LIST[@]}"; do
        MADRONA_BB_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline $mode > "$OUT/tmp.log" 2>&1
        rc=$?
        [ $rc -ne 0 ] && { cat "$OUT/tmp.log"; exit $rc; }
        python3 tools/ab_line.py "$v" "$mode" "$OUT/tmp.log" | tee -a "$OUT/summary.txt"
    done
done
