#!/bin/bash
# Round 5, session ba: the last build (BB_RESIDENT_COL_AUX knob at its
# default) -- every GPU test, smoke and the bench line once more.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05ba tests smoke bench
