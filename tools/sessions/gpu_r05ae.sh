#!/bin/bash
# Round 5, session ae: the staged-step loop with half the workgroups started
# later (sk3a: odd workgroups 3 x s_sleep(127); sk3b: the second half of the
# grid; sk1a: odd, 1 x) -- does an initial phase offset between a CU's two
# workgroups persist and pay?
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r05ae
mkdir -p $OUT
for i in 1 2; do for v in prod sk3a sk3b sk1a; do
    if [ $v = prod ]; then lib=""; else lib=madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/step_loop_sweep.py --worlds 65536,262144,32768 --steps 500 \
        --reps 2 2>&1 | grep -v amdgpu.ids | sed "s|^|$v |" >> $OUT/skew_ab.txt || exit 1
done; done
echo done
