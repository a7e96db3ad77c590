#!/bin/bash
# per-config rocprof kernel stats (one bench workload per run, so each summary's average is that config's kernel)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03ai; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --no-e2e --no-configs "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -20 $O/$tag.log; exit 2; }
  f=$(find $O/$tag -name "*kernel_stats.csv" | head -1); cp $f $O/${tag}_kernel_stats.csv
  grep -h '^{' $O/$tag.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline') or {}; print('$tag', 'events kernel_avg_us', r.get('kernel_avg_us'), 'frac', r.get('frac'))"
  sed -n 2,3p $O/${tag}_kernel_stats.csv | cut -c1-140
}
run W65536_N2 --steps 1000 --warmup 100
run W8192_N2 --worlds 8192 --steps 1000 --warmup 100
run W8192_R32 --worlds 8192 --rollout 32 --steps 1024 --warmup 32
run W65536_N4 --agents 4 --steps 300 --warmup 30
run W65536_N10 --agents 10 --steps 100 --warmup 10
