#!/bin/bash
# Round 5: sessions ag and ah in one call (the pool is congested).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
bash tools/sessions/gpu_r05ag.sh && bash tools/sessions/gpu_r05ah.sh
