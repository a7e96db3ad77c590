#!/bin/bash
# A/B of variant builds on the staged-step sweep (tools/step_loop_sweep.py).
# Usage: WORLDS=32768,65536 KINDS=2 bash tools/ab_sweep.sh <tag> <variant|base>...   (two rounds, interleaved)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib=$ROOT/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 "$ROOT/tools/step_loop_sweep.py" --worlds "${WORLDS:-32768,65536,262144}" \
        --kinds "${KINDS:-2}" --steps "${STEPS:-200}" > "$OUT/tmp.log" 2>&1
    rc=$?
    [ $rc -ne 0 ] && { cat "$OUT/tmp.log"; exit $rc; }
    sed "s/^/$v /" "$OUT/tmp.log" | tee -a "$OUT/summary.txt"
  done
done
