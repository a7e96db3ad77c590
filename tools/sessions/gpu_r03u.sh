#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
timeout -k 10 400 bash tools/pmc_bench.sh r03u/pmc_W65536_N10 --agents 10 --steps 20 --warmup 5 --no-e2e --no-configs || exit 2
timeout -k 10 400 bash tools/pmc_bench.sh r03u/pmc_W65536_N4 --agents 4 --steps 20 --warmup 5 --no-e2e --no-configs || exit 2
