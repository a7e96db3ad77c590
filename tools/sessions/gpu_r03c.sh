set -u
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_policy_rollout.py tests/test_policy_golden.py tests/test_policy.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --worlds 8192 --rollout 32 --policy --steps 640 --warmup 64 --no-cpu-baseline > $O/bench_ppo_8192.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --worlds 65536 --rollout 32 --policy --steps 320 --warmup 32 --no-cpu-baseline > $O/bench_ppo_65536.log 2>&1 || exit $?
timeout -k 10 300 python tools/ablate.py --worlds 8192 --iters 200 --rounds 3 > $O/ablate8k.log 2>&1 || exit $?
timeout -k 10 300 python tools/ablate_systems.py --worlds 8192 --iters 200 > $O/systems8k.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ppo8k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --worlds 8192 --rollout 32 --policy --steps 320 --warmup 32 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_ppo8k.log 2>&1
