#!/bin/bash
# Round 5, session r: PPO A/B -- product (branch-free exp / log, first policy
# pass inside k_rollout_ppo), nopass0 (that pass as a k_policy launch), eb7
# (the build before both changes).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05r
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in 1 2; do for W in 65536 32768 131072 8192; do for v in prod nopass0 eb7; do
    if [ $W = 8192 ] && [ $v = nopass0 ]; then continue; fi
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records.*per_step=0" | sed "s|^|$v $W |" >> $OUT/ppo_ab.txt || exit 1
done; done; done
echo done
