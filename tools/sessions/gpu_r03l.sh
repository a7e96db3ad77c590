set -u
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_rollout.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for r in 1 2; do
for w in 8192 32768 65536 262144; do
  timeout -k 10 200 python tools/ablate.py --worlds $w --iters 200 --rounds 3 --only 0 > $O/base_${w}_$r.log 2>&1 || exit $?
  grep median $O/base_${w}_$r.log | sed "s/^/base W=$w r=$r /" >> $O/summary.txt
  MADRONA_BB_LIB=$PWD/madrona_basketball_amd/_variants/colsc1/libmadrona_basketball_amd.so timeout -k 10 200 python tools/ablate.py --worlds $w --iters 200 --rounds 3 --only 0 > $O/col_${w}_$r.log 2>&1 || exit $?
  grep median $O/col_${w}_$r.log | sed "s/^/colsc1 W=$w r=$r /" >> $O/summary.txt
done
done
