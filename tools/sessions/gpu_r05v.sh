#!/bin/bash
# Round 5, session v: bb_step_n_staged as one k_step_loop launch -- every GPU
# test, the default bench line (headline on the loop kernel, the per-launch
# object beside it), kernel stats of the headline workload.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05v tests bench prof:65536:2 prof:8192:2 prof:262144:2
