#!/bin/bash
# Round 4, final validation of HEAD (last: after the per-part next-value pass
# changes): full pytest -m gpu, smoke, the default bench line, PPO kernel stats
# and PMC passes.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
bash tools/gpu_r04.sh fin4 tests smoke bench profppo:65536 pmcppo:65536
