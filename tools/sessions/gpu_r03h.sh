set -u
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 120 python tools/ppo_trace.py --worlds 8192 > $O/ppo_trace.log 2>&1 || exit $?
timeout -k 10 300 python tools/ablate.py --worlds 65536 --agents 4 --iters 30 --rounds 3 > $O/ablate4.log 2>&1 || exit $?
timeout -k 10 300 python tools/ablate.py --worlds 65536 --agents 10 --iters 10 --rounds 3 > $O/ablate10.log 2>&1 || exit $?
