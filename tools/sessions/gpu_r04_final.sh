#!/bin/bash
# Round 4, final session on the last build: the split PPO's policy kernel at
# 32 768 / 131 072 worlds (k_policy<2> default vs <1>), full pytest -m gpu,
# smoke, the default bench line, and the PPO kernel stats / PMC passes again
# (the PPO path changed after session s1: start-only alignment of the split
# parts, k_policy<2> halves, one threefry call per lane in 16-row bucket passes).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
export PYTHONUNBUFFERED=1
for W in 32768 131072; do
for M in 2 1; do
    MADRONA_BB_PPO_SPLIT_MT=$M timeout -k 10 300 python3 tools/ppo_time.py --worlds $W --rollouts 3 2>&1 | grep -v amdgpu.ids \
        | grep -E "all records" | sed "s|^|W=$W MT=$M |" || exit 1
done
done
bash tools/gpu_r04.sh fin tests smoke bench profppo:65536 pmcppo:65536
