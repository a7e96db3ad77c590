#!/bin/bash
# One gpurun call: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault/abort/timeout (exit >= 124,
# 134, 139, or a signal) ends the script immediately.  Ordinary test failures
# (exit 1) are recorded and the remaining steps still run.
# Usage: bash tools/gpu_round.sh [tag] [steps...]   steps: smoke tests bench prof pmc
set -u
TAG=${1:-r01}
shift || true
STEPS=${*:-smoke tests bench prof}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export PYTHONUNBUFFERED=1

fatal() {  # exit codes that mean the GPU step did not end normally
    local rc=$1
    [ "$rc" -eq 0 ] && return 1
    [ "$rc" -eq 1 ] && return 1   # pytest: tests failed
    [ "$rc" -eq 2 ] && return 1   # pytest: interrupted/usage
    [ "$rc" -eq 5 ] && return 1   # pytest: nothing collected
    return 0
}

run() {  # name timeout cmd...
    local name=$1 tmo=$2
    shift 2
    echo "=== $name ($(date +%T))" | tee -a "$OUT/summary.txt"
    timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a "$OUT/summary.txt"
    tail -n 5 "$OUT/$name.log" | tee -a "$OUT/summary.txt"
    if fatal $rc; then
        echo "FATAL: $name ended with $rc; stopping" | tee -a "$OUT/summary.txt"
        exit $rc
    fi
    return 0
}

for s in $STEPS; do
    case $s in
    smoke) run smoke 420 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread ;;
    bench) run bench 600 python bench.py --steps 1000 --warmup 100 ;;
    rectests) run pytest_recorder 600 python -u -m pytest tests/test_recorder.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    pmcr:*) k=${s#pmcr:}
        ( cd /tmp && export TMPDIR=/tmp && run "pmcr${k}_fetch" 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmcr${k}_fetch" -o run \
            --output-format csv -- python3 "$ROOT/bench.py" --steps $((4*k)) --warmup $k --rollout $k --no-cpu-baseline ) || exit $?
        ( cd /tmp && export TMPDIR=/tmp && run "pmcr${k}_write" 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmcr${k}_write" -o run \
            --output-format csv -- python3 "$ROOT/bench.py" --steps $((4*k)) --warmup $k --rollout $k --no-cpu-baseline ) || exit $?
        python3 tools/traffic.py "$OUT/pmcr${k}_fetch" "$OUT/pmcr${k}_write" W65536_N2_R$k --kernel "k_rollout<2>" \
            --out "$OUT/traffic.json" | tee -a "$OUT/summary.txt"
        ;;
    benchp) run bench_policy 600 python bench.py --steps 300 --warmup 30 --policy --no-cpu-baseline ;;
    profp)
        ( cd /tmp && export TMPDIR=/tmp && run prof_policy 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_policy" -o run \
            --output-format csv -- python3 "$ROOT/bench.py" --steps 200 --warmup 20 --policy --no-cpu-baseline ) || exit $?
        ;;
    rtests) run pytest_rollout 600 python -u -m pytest tests/test_rollout.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    benchr:*) k=${s#benchr:}; run "bench_r$k" 600 python bench.py --steps 1024 --warmup 64 --rollout $k --no-cpu-baseline ;;
    profr:*) k=${s#profr:}
        ( cd /tmp && export TMPDIR=/tmp && run "prof_r$k" 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r$k" -o run \
            --output-format csv -- python3 "$ROOT/bench.py" --steps 512 --warmup 32 --rollout $k --no-cpu-baseline ) || exit $?
        ;;
    bench262k) run bench262k 600 python bench.py --worlds 262144 --steps 300 --warmup 50 --no-cpu-baseline ;;
    bench8k) run bench8k 600 python bench.py --worlds 8192 --steps 1000 --warmup 100 --no-cpu-baseline ;;
    bench4) run bench4 600 python bench.py --agents 4 --steps 300 --warmup 50 --no-cpu-baseline ;;
    bench10) run bench10 600 python bench.py --agents 10 --steps 100 --warmup 20 --no-cpu-baseline ;;
    ablate) run ablate 600 python tools/ablate.py --worlds 65536 ;;
    ablate262k) run ablate262k 600 python tools/ablate.py --worlds 262144 --iters 50 ;;
    ablate4) run ablate4 600 python tools/ablate.py --worlds 65536 --agents 4 --iters 30 --rounds 3 ;;
    ablate10) run ablate10 600 python tools/ablate.py --worlds 65536 --agents 10 --iters 10 --rounds 3 ;;
    systems) run systems 600 python tools/ablate_systems.py --worlds 65536 ;;
    pmcab) run pmcab 900 bash tools/pmc_ablate.sh "$TAG/pmc" 65536 ;;
    prof)
        ( cd /tmp && export TMPDIR=/tmp && run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
            --output-format csv -- python3 "$ROOT/bench.py" --steps 300 --warmup 30 --no-cpu-baseline ) || exit $?
        ;;
    pmc)
        ( cd /tmp && export TMPDIR=/tmp && run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run \
            --output-format csv -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline ) || exit $?
        ( cd /tmp && export TMPDIR=/tmp && run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run \
            --output-format csv -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline ) || exit $?
        python3 tools/traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" W65536_N2 --out "$OUT/traffic.json" | tee -a "$OUT/summary.txt"
        ;;
    pmcx:*) v=${s#pmcx:}; w=${v%%:*}; n=${v#*:}  # pmcx:<worlds>:<agents>, k_step<n> traffic per launch
        for c in FETCH_SIZE WRITE_SIZE; do
            ( cd /tmp && export TMPDIR=/tmp && run "pmc_W${w}_N${n}_$c" 300 rocprofv3 --pmc $c \
                -d "$OUT/pmc_W${w}_N${n}_$c" -o run --output-format csv -- python3 "$ROOT/bench.py" \
                --worlds $w --agents $n --steps 20 --warmup 5 --no-cpu-baseline --no-e2e ) || exit $?
        done
        python3 tools/traffic.py "$OUT/pmc_W${w}_N${n}_FETCH_SIZE" "$OUT/pmc_W${w}_N${n}_WRITE_SIZE" W${w}_N${n} \
            --kernel "k_step<$n, 0," --out "$OUT/traffic.json" | tee -a "$OUT/summary.txt"
        ;;
    profx:*) v=${s#profx:}; w=${v%%:*}; n=${v#*:}  # profx:<worlds>:<agents>: kernel stats of that bench line
        ( cd /tmp && export TMPDIR=/tmp && run "prof_W${w}_N${n}" 600 rocprofv3 --kernel-trace --stats \
            -d "$OUT/prof_W${w}_N${n}" -o run --output-format csv -- python3 "$ROOT/bench.py" \
            --worlds $w --agents $n --steps 200 --warmup 20 --no-cpu-baseline --no-e2e ) || exit $?
        ;;
    benchrw:*) v=${s#benchrw:}; w=${v%%:*}; k=${v#*:}  # benchrw:<worlds>:<K>: rollouts of K steps
        run "bench_W${w}_R$k" 600 python bench.py --worlds $w --rollout $k --steps $((32*k)) --warmup $k --no-cpu-baseline ;;
    benchx:*) v=${s#benchx:}; w=${v%%:*}; n=${v#*:}
        run "bench_W${w}_N${n}" 600 python bench.py --worlds $w --agents $n --steps 300 --warmup 30 --no-cpu-baseline ;;
    pmcv:*) v=${s#pmcv:}
        for c in FETCH_SIZE WRITE_SIZE; do
            ( cd /tmp && export TMPDIR=/tmp && \
              MADRONA_BB_LIB=$ROOT/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so \
              run "pmc_${v}_$c" 300 rocprofv3 --pmc $c -d "$OUT/pmc_${v}_$c" -o run --output-format csv -- \
                python3 "$ROOT/tools/ablate.py" --worlds 65536 --iters 20 --rounds 1 --only 0 ) || exit $?
        done ;;
    abn:*) v=${s#abn:}; n=${v#*:}; v=${v%%:*}
        MADRONA_BB_LIB=$ROOT/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so \
            run "ablate_${v}_n$n" 600 python tools/ablate.py --worlds 65536 --agents $n --iters 10 --rounds 3 --only 0 1 2 4 ;;
    ab:*) v=${s#ab:}
        MADRONA_BB_LIB=$ROOT/madrona_basketball_amd/_variants/$v/libmadrona_basketball_amd.so \
            run "ablate_$v" 600 python tools/ablate.py --worlds 65536 ;;
    *) echo "unknown step $s" ;;
    esac
done
echo "=== done" | tee -a "$OUT/summary.txt"
