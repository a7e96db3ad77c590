#!/bin/bash
# Round-5/6 GPU session steps.  One rocprofv3 run per workload (kernel stats of
# one configuration alone), PMC passes one counter group per run.  Every GPU
# step has its own time limit; the first failing step ends the script.
# Usage: bash tools/gpu_r05.sh <tag> <step>...
#   bench                      default bench line (all configs, CPU baselines)
#   benchshort                 the driver's invocation (--gpus 1 --steps 20 --warmup 5)
#   prof:<W>:<N>               kernel stats of k_step<N> at W worlds, that workload alone
#   profhead                   kernel stats of the headline line's own command (default steps)
#   profppo:<W>                kernel stats of the PPO rollout (K=32) at W worlds
#   profro:<W>:<K>[:<N>]       kernel stats of bb_rollout (K steps per launch) at W worlds (N agents)
#   pmc:<W>:<N>                FETCH_SIZE / WRITE_SIZE of k_step<N> (two passes)
#   pmcppo:<W>                 FETCH_SIZE / WRITE_SIZE of the PPO rollout's kernels
#   pmcro:<W>:<K>[:<N>]        FETCH_SIZE / WRITE_SIZE of bb_rollout
#   sqppo:<W>                  SQ counters of the PPO rollout's kernels (K=32)
#   sq:<W>:<N>                 SQ issue / wait / instruction counters of k_step<N>
#   pmcl:<W>:<N> / sql:<W>:<N> the same of the staged-step loop (200-step launches)
#   tests                      pytest -m gpu
#   pytest:<file>[:<k expr>]   pytest -m gpu of one test file (optionally -k)
#   smoke                      __graft_entry__.smoke()
#   py:<file>                  python <file> (a diagnostic script under tools/)
set -u
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-configs"

step() {  # name timeout cmd...
    local name=$1 tmo=$2
    shift 2
    echo "=== $name $(date +%T)"
    (cd /tmp && TMPDIR=/tmp timeout -k 10 "$tmo" "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 3 "$OUT/$name.log"
    [ $rc -eq 0 ] || { echo "FATAL: $name rc=$rc"; exit $rc; }
}

SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"

for s in "$@"; do
    IFS=: read -r kind a b c <<< "$s"
    n=${c:-2}; sfx=${c:+_N$c}
    case $kind in
    bench) step bench 600 python3 "$R/bench.py" --steps 1000 --warmup 100 ;;
    benchshort) step bench_short 600 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 ;;
    tests) step pytest_gpu 900 python3 -u -m pytest "$R/tests" -m gpu -q -rfE --timeout 300 --timeout-method thread ;;
    pytest) if [ -n "$b" ]; then
                step "pytest_$(basename "$a" .py)" 600 python3 -u -m pytest "$R/$a" -m gpu -q -rfE -k "$b" --timeout 240 --timeout-method thread
            else
                step "pytest_$(basename "$a" .py)" 600 python3 -u -m pytest "$R/$a" -m gpu -q -rfE --timeout 240 --timeout-method thread
            fi ;;
    smoke) step smoke 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" ;;
    prof) step "prof_W${a}_N$b" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_W${a}_N$b" -o run --output-format csv \
            -- $B --worlds "$a" --agents "$b" --steps 300 --warmup 30 ;;
    profhead) step prof_headline 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_headline" -o run --output-format csv \
            -- python3 "$R/bench.py" --no-cpu-baseline --no-e2e --no-configs ;;
    profppo) step "prof_ppo_W$a" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_ppo_W$a" -o run --output-format csv \
            -- $B --worlds "$a" --policy --rollout 32 --steps 320 --warmup 32 ;;
    profro) step "prof_ro_W${a}_R$b$sfx" 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_ro_W${a}_R$b$sfx" -o run \
            --output-format csv -- $B --worlds "$a" --agents "$n" --rollout "$b" --steps $((16 * b)) --warmup "$b" ;;
    pmc) for c in FETCH_SIZE WRITE_SIZE; do
            step "pmc_W${a}_N${b}_$c" 120 rocprofv3 --pmc $c -d "$OUT/pmc_W${a}_N${b}_$c" -o run --output-format csv \
                -- $B --worlds "$a" --agents "$b" --steps 20 --warmup 5
         done ;;
    pmcl) for c in FETCH_SIZE WRITE_SIZE; do  # the staged-step loop: 200-step launches
            step "pmcl_W${a}_N${b}_$c" 180 rocprofv3 --pmc $c -d "$OUT/pmcl_W${a}_N${b}_$c" -o run --output-format csv \
                -- $B --worlds "$a" --agents "$b" --steps 200 --warmup 5
         done ;;
    sql) step "sql_W${a}_N$b" 180 rocprofv3 --pmc $SQ -d "$OUT/sql_W${a}_N$b" -o run --output-format csv \
            -- $B --worlds "$a" --agents "$b" --steps 200 --warmup 5 ;;
    pmcppo) for c in FETCH_SIZE WRITE_SIZE; do
            step "pmc_ppo_W${a}_$c" 120 rocprofv3 --pmc $c -d "$OUT/pmc_ppo_W${a}_$c" -o run --output-format csv \
                -- $B --worlds "$a" --policy --rollout 32 --steps 64 --warmup 32
         done ;;
    pmcro) for ctr in FETCH_SIZE WRITE_SIZE; do
            step "pmc_ro_W${a}_R${b}${sfx}_$ctr" 120 rocprofv3 --pmc $ctr -d "$OUT/pmc_ro_W${a}_R${b}${sfx}_$ctr" -o run \
                --output-format csv -- $B --worlds "$a" --agents "$n" --rollout "$b" --steps $((2 * b)) --warmup "$b"
         done ;;
    sqppo) step "sq_ppo_W$a" 120 rocprofv3 --pmc $SQ -d "$OUT/sq_ppo_W$a" -o run --output-format csv \
            -- $B --worlds "$a" --policy --rollout 32 --steps 64 --warmup 32 ;;
    sq) step "sq_W${a}_N$b" 120 rocprofv3 --pmc $SQ -d "$OUT/sq_W${a}_N$b" -o run --output-format csv \
            -- $B --worlds "$a" --agents "$b" --steps 20 --warmup 5 ;;
    py) step "py_$(basename "$a" .py)${b:+_${b//[^A-Za-z0-9]/}}" 600 python3 "$R/$a" ${b//,/ } ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "=== done"
