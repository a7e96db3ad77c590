#!/bin/bash
# Round 4, session s2 (final build): full pytest -m gpu, smoke, the default
# bench line (every config, CPU baselines), a 2-rank gloo rehearsal of the
# multi-rank bench path on the one GPU, and the N = 10 trace of tools/ablate.py.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r04.sh s2 tests smoke bench "py:tools/ablate.py:--worlds 65536 --agents 10 --iters 20 --rounds 3" || exit $?
OUT=$R/gpurun_out/s2
echo "=== dist2 $(date +%T)"
(cd /tmp && TMPDIR=/tmp timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 "$R/bench.py" --gpus 2 --dist-backend gloo --steps 300 --warmup 30 \
    --no-cpu-baseline) > $OUT/dist2_gloo.log 2>&1
rc=$?; echo "=== dist2 rc=$rc"; tail -c 600 $OUT/dist2_gloo.log; exit $rc
