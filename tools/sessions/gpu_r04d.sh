#!/bin/bash
# Round 4, session d: policy kernel shapes at 65 536 rows (MT, persistent grid).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
OUT=gpurun_out/d
mkdir -p $OUT
export PYTHONUNBUFFERED=1 MADRONA_BB_POLICY_ROWS=0
for cfg in "1 0" "1 1024" "1 2048" "1 3072" "2 0" "2 1024" "2 2048" "4 0" "4 512"; do
    set -- $cfg
    if [ "$2" = 0 ]; then unset MADRONA_BB_POLICY_GRID; else export MADRONA_BB_POLICY_GRID=$2; fi
    echo "MT=$1 GRID=$2"
    MADRONA_BB_POLICY_MT=$1 timeout -k 10 120 python3 tools/policy_time.py --worlds 65536 2>&1 | grep -v amdgpu.ids | grep "agent 0" || exit 1
done
bash tools/sessions/gpu_r04e.sh
