#!/bin/bash
# Round-3: PMC of k_step<4> / k_step<10> at 65 536 worlds after the row-pass
# change -- HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and one SQ
# pass (issue vs waits) per N.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/ay
mkdir -p $OUT
for n in 4 10; do
  for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
    tag=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmc_n${n}_$tag -o run --output-format csv -- \
      python3 $R/bench.py --worlds 65536 --agents $n --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-configs \
      > $OUT/pmc_n${n}_$tag.log 2>&1 || { echo "pmc n$n $tag failed rc=$?"; exit 1; }
    echo "pmc n$n $tag ok"
  done
done
echo done
