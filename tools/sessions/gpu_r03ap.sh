#!/bin/bash
# Round-3 A/B: emit_pieces read batches (product) vs row-by-row (variant rb1)
# at N = 4 / 10; k_policy_wg with 12 (product) vs 16 (variant pwg16) waves per
# workgroup vs the register-weight k_policy.  Parity first.
set -u
OUT=gpurun_out/ap
mkdir -p $OUT
V=$PWD/madrona_basketball_amd/_variants
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 2 $OUT/$n.log; [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_reference_math.py tests/test_policy.py tests/test_policy_rollout.py -m gpu -x -q --timeout 120 --timeout-method thread
for n in 4 10; do
  step ab_n${n}_rb 300 python tools/ablate.py --worlds 65536 --agents $n --iters 20 --rounds 3 --only 0 2
  MADRONA_BB_LIB=$V/rb1/libmadrona_basketball_amd.so step ab_n${n}_rb1 300 python tools/ablate.py --worlds 65536 --agents $n --iters 20 --rounds 3 --only 0 2
done
step ab_n4_8k_rb 300 python tools/ablate.py --worlds 8192 --agents 4 --iters 50 --rounds 3 --only 0
MADRONA_BB_LIB=$V/rb1/libmadrona_basketball_amd.so step ab_n4_8k_rb1 300 python tools/ablate.py --worlds 8192 --agents 4 --iters 50 --rounds 3 --only 0
step pol_wg12 200 python tools/policy_time.py --trace
MADRONA_BB_LIB=$V/pwg16/libmadrona_basketball_amd.so step pol_wg16 200 python tools/policy_time.py --trace
MADRONA_BB_POLICY_WG=0 step pol_old 200 python tools/policy_time.py
echo done
