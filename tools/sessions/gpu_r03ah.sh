#!/bin/bash
# k_policy tile shape x grid cap (persistent waves with next-tile prefetch)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03ah; mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_policy.py tests/test_policy_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "4 0" "1 0" "1 1024" "2 1024" "4 1024" "1 512" "4 512"; do
  set -- $cfg
  MADRONA_BB_POLICY_MT=$1 MADRONA_BB_POLICY_GRID=$2 timeout -k 10 120 python tools/policy_time.py --worlds 65536 --iters 50 > $O/p_mt$1_g$2.log 2>&1 || { tail -5 $O/p_mt$1_g$2.log; exit 2; }
  grep "rows" $O/p_mt$1_g$2.log | sed "s/^/MT=$1 grid=$2 /"
done
