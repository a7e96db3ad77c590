#!/bin/bash
# list the gfx950 counters that mention instruction fetch / icache
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r03ac; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -i -E "icache|ifetch|SQC_|INST_LEVEL|WAIT_INST|SQ_INSTS_" $O/avail.txt | head -80 > $O/icache_counters.txt || true
wc -l $O/avail.txt $O/icache_counters.txt
