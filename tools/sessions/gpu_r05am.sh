#!/bin/bash
# Round 5, session am: the register-resident staged loop (bb_step_n_staged at
# 2 agents up to one wave per SIMD) -- bench line, every GPU test, smoke,
# kernel stats and PMC traffic of the C2 / C4 workloads, the headline profile.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05am bench tests smoke prof:8192:2 prof:32768:2 profhead pmcl:8192:2 pmcl:32768:2
