#!/bin/bash
# Round 6, session g: evidence of this round's build -- the headline's
# rocprof (its own command), PMC traffic of the resident loop and of one
# k_step per step (the per-call object), of the PPO rollouts (against the
# fused step's new algorithmic bytes), and bench.py --gpus 2 starting its own
# two ranks (gloo, both on the one GPU: a rehearsal of the line's shape).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
bash "$R/tools/gpu_r06.sh" r06g profhead pmcl:65536:2 pmcppo:65536 pmcppo:8192 || exit $?
OUT=$R/gpurun_out/r06g
timeout -k 10 400 python3 "$R/bench.py" --gpus 2 --steps 100 --warmup 10 --dist-backend gloo --no-cpu-baseline \
    > $OUT/bench_gpus2_self.json 2> $OUT/bench_gpus2_self.log || exit $?
echo done
