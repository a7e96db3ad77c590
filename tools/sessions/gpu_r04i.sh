#!/bin/bash
# Round 4, session i: SQ counters and phase traces of k_policy<4> / <2> at 65 536 rows.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=$R/gpurun_out/i
mkdir -p $OUT
bash tools/sessions/gpu_r04j.sh || exit 1
export PYTHONUNBUFFERED=1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
SQ2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC"
for mt in 4 2; do
  for set in SQ SQ2; do
    (cd /tmp && MADRONA_BB_POLICY_MT=$mt timeout -s KILL 90 rocprofv3 --pmc ${!set} -d $OUT/pmc_mt${mt}_$set -o run --output-format csv \
        -- python3 $R/tools/policy_time.py --worlds 65536 --only-argmax --iters 20) > $OUT/pmc_mt${mt}_$set.log 2>&1 || { tail -5 $OUT/pmc_mt${mt}_$set.log; exit 1; }
  done
  MADRONA_BB_POLICY_MT=$mt timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 --trace --only-argmax 2>&1 | grep -v amdgpu.ids | sed "s|^|MT$mt |" || exit 1
done
echo done
