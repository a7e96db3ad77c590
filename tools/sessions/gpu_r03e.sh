set -u
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_policy_rollout.py tests/test_policy_golden.py tests/test_policy.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for mt in 1 2 4; do
  MADRONA_BB_POLICY_MT=$mt timeout -k 10 300 python tools/policy_time.py --worlds 65536 > $O/policy_time_mt$mt.log 2>&1 && MADRONA_BB_POLICY_MT=$mt timeout -k 10 300 python tools/policy_time.py --worlds 8192 >> $O/policy_time_mt$mt.log 2>&1 || exit $?
  MADRONA_BB_POLICY_MT=$mt timeout -k 10 300 python bench.py --worlds 8192 --rollout 32 --policy --steps 640 --warmup 64 --no-cpu-baseline > $O/bench_ppo_8192_mt$mt.log 2>&1 || exit $?
  MADRONA_BB_POLICY_MT=$mt timeout -k 10 300 python bench.py --worlds 65536 --rollout 32 --policy --steps 320 --warmup 32 --no-cpu-baseline > $O/bench_ppo_65536_mt$mt.log 2>&1 || exit $?
done
