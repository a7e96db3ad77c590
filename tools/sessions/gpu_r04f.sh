#!/bin/bash
# Round 4, session f: buffer.obs record as whole-line stores (LDS-staged) vs
# per-lane; 16-wave policy workgroups.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/f
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
V=$R/madrona_basketball_amd/_variants
for rep in 1 2; do
for lib in "" $V/recreg/libmadrona_basketball_amd.so; do
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds 65536 \
        --policy --rollout 32 --steps 320 --warmup 32 > $OUT/ppo.log 2>&1 || exit $?
    python3 -c "import json;d=[json.loads(l) for l in open('$OUT/ppo.log') if l.startswith('{')][-1];print('${lib:-product}'[-40:], 'PPO 65536', round(d['value']/1e9,3), 'G/s', round(d['policy_rollout']['us_per_step'],2), 'us/step')"
done
done
for lib in "" $V/pwg16/libmadrona_basketball_amd.so; do
    MADRONA_BB_POLICY_WG=1 MADRONA_BB_LIB=$lib timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | grep "agent 0" | sed "s|^|${lib:-product12} |" || exit 1
done
