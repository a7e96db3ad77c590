#!/bin/bash
# SQ / traffic counters of the bench workload, one counter group per rocprofv3
# pass (no trace domains combined with --pmc).  Extra bench.py args after the tag.
# Usage: bash tools/pmc_bench.sh <tag> [bench args...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-pmc}
shift || true
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/g$i" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/g$i.log" 2>&1
    rc=$?
    echo "group $i ($grp) rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" | tee "$OUT/summary.txt"
exit 0
