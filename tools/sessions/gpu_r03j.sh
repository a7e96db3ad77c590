set -u
O=gpurun_out/r03j; mkdir -p $O
V=$PWD/madrona_basketball_amd/_variants/parts1/libmadrona_basketball_amd.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_math.py tests/test_gpu_scenarios.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2; do
for cfg in "65536 4" "262144 4" "8192 4"; do
  set -- $cfg
  timeout -k 10 200 python tools/ablate.py --worlds $1 --agents $2 --iters 50 --rounds 3 --only 0 > $O/new_$1_$2_$r.log 2>&1 || exit $?
  grep median $O/new_$1_$2_$r.log | sed "s/^/new W=$1 N=$2 r=$r /" >> $O/summary.txt
  MADRONA_BB_LIB=$V timeout -k 10 200 python tools/ablate.py --worlds $1 --agents $2 --iters 50 --rounds 3 --only 0 > $O/old_$1_$2_$r.log 2>&1 || exit $?
  grep median $O/old_$1_$2_$r.log | sed "s/^/old W=$1 N=$2 r=$r /" >> $O/summary.txt
done
done
timeout -k 10 300 python tools/ablate.py --worlds 65536 --agents 4 --iters 30 --rounds 2 > $O/trace4_new.log 2>&1 || exit $?
