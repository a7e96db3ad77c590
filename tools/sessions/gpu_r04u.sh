#!/bin/bash
# Round 4, session u: cache policy of the PPO buffer.obs record stores
# (BB_REC_AUX: nt = product, plain, sc1), split per-step PPO at 65 536 worlds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
V=$R/madrona_basketball_amd/_variants
for i in 1 2; do
for v in base recplain recsc1; do
    if [ $v = base ]; then lib=""; else lib=$V/$v/libmadrona_basketball_amd.so; fi
    MADRONA_BB_LIB=$lib timeout -k 10 300 python3 tools/ppo_time.py --worlds 65536 --rollouts 4 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records|value" | sed "s|^|$v |" || exit 1
done
done
