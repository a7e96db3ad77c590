#!/bin/bash
# Round 5, session s: sessions q and r in one call (the pool is congested).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
bash tools/sessions/gpu_r05q.sh && bash tools/sessions/gpu_r05r.sh
