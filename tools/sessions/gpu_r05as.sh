#!/bin/bash
# Round 5, session as: the resident staged loop at every agent count (shared-
# world instances while the step stays in the Infinity Cache) -- bench line,
# every GPU test, smoke, kernel stats and PMC traffic of the new launches.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r05.sh" r05as bench tests smoke profhead prof:65536:4 prof:65536:10 pmcl:65536:4
