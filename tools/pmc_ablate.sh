#!/bin/bash
# PMC counters per k_step variant (each variant is its own kernel symbol).
# One counter group per rocprofv3 pass (no trace domains combined with --pmc).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-pmc}
W=${2:-65536}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/g$i" -o run --output-format csv -- \
        python3 "$ROOT/tools/ablate.py" --worlds $W --iters 20 --rounds 1 > "$OUT/g$i.log" 2>&1
    rc=$?
    echo "group $i ($grp) rc=$rc"
    [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
