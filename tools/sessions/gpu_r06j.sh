#!/bin/bash
# Round 6, session j: the maximum-size tests (4 194 304 worlds), and SQ
# counters of this round's headline (resident loop) and per-call (k_step)
# kernels at 65 536 x 2.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r06.sh" r06j pytest:tests/test_gpu_headline.py sql:65536:2 sq:65536:2 || exit $?
echo done
