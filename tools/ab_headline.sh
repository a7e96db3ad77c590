#!/bin/bash
# A/B of variant builds on the headline line (bench.py defaults, no CPU
# baseline / e2e / configs), interleaved ROUNDS times.
# Usage: ROUNDS=3 bash tools/ab_headline.sh <tag> <variant|base>...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for round in $(seq "${ROUNDS:-3}"); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib=$ROOT/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline --no-e2e --no-configs ${BENCH_ARGS:-} > "$OUT/tmp.log" 2>&1
    rc=$?
    [ $rc -ne 0 ] && { cat "$OUT/tmp.log"; exit $rc; }
    python3 "$ROOT/tools/ab_line.py" "$v" "${BENCH_ARGS:-default}" "$OUT/tmp.log" | tee -a "$OUT/summary.txt"
  done
done
