#!/bin/bash
# Round 6, session a: baseline of this round's box -- the default bench line
# (every config) and the rocprof kernel summary of the headline run.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
OUT=gpurun_out/r06a
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-configs --no-e2e \
    > $OUT/prof_bench.json 2> $OUT/prof.log || exit 1
echo done
