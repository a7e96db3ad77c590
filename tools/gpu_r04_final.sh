#!/bin/bash
# Round 4, final session on the last build: full pytest -m gpu, smoke, the
# default bench line, and the PPO kernel stats / PMC passes again (the PPO
# path changed after session s1: start-only alignment of the split parts,
# one threefry call per lane in 16-row bucket passes).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r04.sh fin tests smoke bench profppo:65536 pmcppo:65536
