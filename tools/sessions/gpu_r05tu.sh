#!/bin/bash
# Round 5: sessions t and u in one call.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
bash tools/sessions/gpu_r05t.sh && bash tools/sessions/gpu_r05u.sh
