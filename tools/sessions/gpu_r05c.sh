#!/bin/bash
# Round 5, session c: (1) where a k_step_ppo launch's time goes at 65 536 and
# 32 768 worlds (per-wave phase clocks + parts left out); (2) the buffer.obs
# record's cache policy (nt, plain, sc1) in A/B; (3) the 8 192-world fused PPO
# rollout's per-step trace at HEAD.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05c
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 tools/ppo_step_trace.py --worlds 65536 > $OUT/pps_trace_W65536.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/ppo_step_trace.py --worlds 32768 --no-ablate > $OUT/pps_trace_W32768.log 2>&1 || exit $?
for i in 1 2; do
for v in nt rec_plain rec_sc1; do
    if [ $v = nt ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "per_step=0" | sed "s|^|$v |" >> $OUT/rec_policy_ab.txt || exit 1
done
done
timeout -k 10 300 python3 tools/ppo_trace.py --worlds 8192 > $OUT/ppo_trace_W8192.log 2>&1 || exit $?
echo done
