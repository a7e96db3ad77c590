#!/bin/bash
# Round 5, session ax: SQ counters of the resident staged loop (headline and
# C2 sizes) for DESIGN §10's where-the-time-goes reading.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05ax sql:65536:2 sql:8192:2 sql:32768:2
