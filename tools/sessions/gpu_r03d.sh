set -u
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_math.py tests/test_gpu_scenarios.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools/ablate.py --worlds 8192 --iters 200 --rounds 3 --only 0 > $O/ablate8k_wide.log 2>&1 || exit $?
timeout -k 10 300 python tools/ablate.py --worlds 8192 --iters 200 --rounds 3 > $O/ablate8k_wide_trace.log 2>&1 || exit $?
MADRONA_BB_WIDE_MAX_WAVES=0 timeout -k 10 300 python tools/ablate.py --worlds 8192 --iters 200 --rounds 3 --only 0 > $O/ablate8k_base.log 2>&1 || exit $?
for w in 4096 16384 32768; do
  timeout -k 10 300 python tools/ablate.py --worlds $w --iters 200 --rounds 3 --only 0 > $O/ablate${w}_wide.log 2>&1 || exit $?
  MADRONA_BB_WIDE_MAX_WAVES=0 timeout -k 10 300 python tools/ablate.py --worlds $w --iters 200 --rounds 3 --only 0 > $O/ablate${w}_base.log 2>&1 || exit $?
done
