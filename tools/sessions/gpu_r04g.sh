#!/bin/bash
# Round 4, session g: inverse-CDF sampling (all policy kernels vs the host),
# policy kernel timings at 65 536 rows, PPO lines.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/g
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py tests/test_policy_wg.py \
    tests/test_policy_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
V=$R/madrona_basketball_amd/_variants
timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | sed "s|^|MT4 |" || exit 1
MADRONA_BB_POLICY_WG=1 timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | sed "s|^|WG12 |" || exit 1
MADRONA_BB_POLICY_WG=1 MADRONA_BB_LIB=$V/pwg16/libmadrona_basketball_amd.so timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | sed "s|^|WG16 |" || exit 1
for args in "" "MADRONA_BB_POLICY_WG=1" "MADRONA_BB_POLICY_WG=1 MADRONA_BB_LIB=$V/pwg16/libmadrona_basketball_amd.so"; do
  for W in 65536 8192; do
    env $args timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --no-configs --worlds $W \
        --policy --rollout 32 --steps 320 --warmup 32 > $OUT/ppo.log 2>&1 || exit $?
    python3 -c "import json;d=[json.loads(l) for l in open('$OUT/ppo.log') if l.startswith('{')][-1];print('${args##*/}'[-30:] or 'default', 'PPO $W', round(d['value']/1e9,3), 'G/s', round(d['policy_rollout']['us_per_step'],2), 'us/step')"
  done
done
