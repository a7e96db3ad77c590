set -u
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_policy_rollout.py tests/test_policy_golden.py tests/test_policy.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 120 python tools/ppo_trace.py --worlds 8192 > $O/ppo_trace.log 2>&1 || exit $?
for w in 8192 16384; do
timeout -k 10 300 python bench.py --worlds $w --rollout 32 --policy --steps 640 --warmup 64 --no-cpu-baseline > $O/bench_ppo_${w}_fused.log 2>&1 || exit $?
done
