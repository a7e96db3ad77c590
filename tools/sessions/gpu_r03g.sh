set -u
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_policy_rollout.py tests/test_policy_golden.py tests/test_policy.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --worlds 8192 --rollout 32 --policy --steps 640 --warmup 64 --no-cpu-baseline > $O/bench_ppo_8192_fused.log 2>&1 || exit $?
MADRONA_BB_PPO_FUSED_MAX_WORLDS=0 timeout -k 10 300 python bench.py --worlds 8192 --rollout 32 --policy --steps 640 --warmup 64 --no-cpu-baseline > $O/bench_ppo_8192_unfused.log 2>&1 || exit $?
MADRONA_BB_PPO_FUSED_MAX_WORLDS=65536 timeout -k 10 300 python bench.py --worlds 65536 --rollout 32 --policy --steps 320 --warmup 32 --no-cpu-baseline > $O/bench_ppo_65536_fused.log 2>&1 || exit $?
MADRONA_BB_PPO_FUSED_MAX_WORLDS=32768 timeout -k 10 300 python bench.py --worlds 16384 --rollout 32 --policy --steps 320 --warmup 32 --no-cpu-baseline > $O/bench_ppo_16384_fused.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --worlds 16384 --rollout 32 --policy --steps 320 --warmup 32 --no-cpu-baseline > $O/bench_ppo_16384_unfused.log 2>&1 || exit $?
