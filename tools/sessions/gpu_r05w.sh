#!/bin/bash
# Round 5, session w: session v's bench and kernel stats after the event fix
# (the loop launch's stop event was never waited on).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05w pytest:tests/test_gpu_parity.py:staged bench prof:65536:2 prof:8192:2 prof:262144:2 prof:32768:2
