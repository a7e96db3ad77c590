#!/bin/bash
# Round 5, session ah: k_rollout_ppo with the workgroup's 8 waves kept in
# step by a barrier per step (ppobar) vs free drift.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05ah
mkdir -p $OUT
for i in 1 2; do for W in 65536 32768 131072; do for v in prod ppobar; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records.*per_step=0" | sed "s|^|$v $W |" >> $OUT/ppobar_ab.txt || exit 1
done; done; done
echo done
