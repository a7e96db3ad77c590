set -u
O=gpurun_out/r03n; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ppo8k -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --worlds 8192 --rollout 32 --policy --steps 320 --warmup 32 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_ppo8k.log 2>&1
