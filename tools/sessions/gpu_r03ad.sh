#!/bin/bash
# instruction-cache counters of k_step<2> (8192 and 65536 worlds) and the fused PPO rollout (8192)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r03ad; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "--worlds 8192 --steps 200 --warmup 20" "--worlds 65536 --steps 200 --warmup 20" "--worlds 8192 --rollout 32 --policy --steps 64 --warmup 0"; do
  for grp in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH SQ_WAVES" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/g$i" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --no-cpu-baseline --no-e2e --no-configs $cfg > "$OUT/g$i.log" 2>&1
    rc=$?
    echo "group $i ($cfg | $grp) rc=$rc"
    [ $rc -ne 0 ] && exit $rc
    python3 "$ROOT/tools/pmc_summary.py" "$OUT/g$i" | tee -a "$OUT/summary.txt"
  done
done
exit 0
