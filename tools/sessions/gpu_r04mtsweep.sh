#!/bin/bash
# Round 4: standalone policy pass (FusedPolicy.act) row-count threshold of the
# register-weight kernel: k_policy<1/2/4> at 16 384 ... 65 536 rows.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
for W in 16384 24576 32768 49152; do
for M in 1 2 4; do
    MADRONA_BB_POLICY_MT=$M timeout -k 10 120 python3 tools/policy_time.py --worlds $W 2>&1 | grep -v amdgpu.ids \
        | sed "s|^|MT$M |" || exit 1
done
done
