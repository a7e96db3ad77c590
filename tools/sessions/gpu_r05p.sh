#!/bin/bash
# Round 5, session p: branch-free policy exp / log and bucket loops, the first
# policy pass inside k_rollout_ppo, the N = 4 rollout's mirror as a second
# store -- every GPU test, then PPO timings, the N = 4 rollout line, traces.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05p
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1
rc=$?; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for W in 65536 32768 8192 16384; do
    timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "per_step=0" | sed "s|^|$W |" >> $OUT/ppo_time.txt || exit 1
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds 65536 --agents 4 --rollout 32 \
    --steps 320 --warmup 32 > $OUT/bench_ro32_W65536_N4.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/policy_time.py --worlds 65536 > $OUT/policy_time_W65536.txt 2>&1 || exit $?
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192.txt 2>&1 || exit $?
timeout -k 10 400 python3 tools/ppo_step_trace.py --worlds 65536 > $OUT/pps_trace_W65536.txt 2>&1 || exit $?
echo done
