#!/bin/bash
# Round 5, session y: k_step_loop with workgroups of 4 / 8 waves kept in step
# by a barrier after every step (lg4, lg8) against the 1-wave loop.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r05y
for v in prod lg4 lg8; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/step_loop_sweep.py --worlds 8192,32768,65536,131072,262144 \
        2>&1 | grep -v amdgpu.ids | sed "s|^|$v |" >> gpurun_out/r05y/sweep.txt || exit 1
done
echo done
