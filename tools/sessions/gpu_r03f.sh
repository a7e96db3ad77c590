set -u
O=gpurun_out/r03f; mkdir -p $O
for mt in 1 4; do
  MADRONA_BB_POLICY_MT=$mt timeout -k 10 300 python tools/policy_time.py --worlds 8192 --trace --only-argmax --iters 5 > $O/trace8k_mt$mt.log 2>&1 || exit $?
  MADRONA_BB_POLICY_MT=$mt timeout -k 10 300 python tools/policy_time.py --worlds 65536 --trace --only-argmax --iters 5 > $O/trace65k_mt$mt.log 2>&1 || exit $?
done
