#!/bin/bash
# Round 4, final validation of HEAD (after the bucket-noise and pol_select
# changes): full pytest -m gpu, smoke, the default bench line, PPO kernel stats
# and PMC passes.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
bash tools/gpu_r04.sh fin2 tests smoke bench profppo:65536 pmcppo:65536
