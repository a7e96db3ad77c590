#!/bin/bash
# Round 4: PPO per-step loop with the trainee's rows written into buffer.obs
# only (the policy reads them there) vs also into the sim's obs; parity first.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
mkdir -p gpurun_out/ro
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_policy_rollout.py tests/test_policy.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/ro/pytest.log 2>&1
rc=$?; echo "tests: $(tail -n 1 gpurun_out/ro/pytest.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/ro/pytest.log; exit $rc; }
for i in 1 2; do
for v in 1 0; do
for W in 65536 32768; do
    MADRONA_BB_PPO_REC_ONLY=$v timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records" | sed "s|^|rec_only=$v W=$W |" || exit 1
done
done
done
