set -u
O=gpurun_out/r03i; mkdir -p $O
V=$PWD/madrona_basketball_amd/_variants/erf_glob/libmadrona_basketball_amd.so
true
for r in 1 2; do
for w in 8192 65536 262144; do
  timeout -k 10 200 python tools/ablate.py --worlds $w --iters 200 --rounds 3 --only 0 > $O/new_${w}_${r}.log 2>&1 || exit $?
  grep median $O/new_${w}_${r}.log | sed "s/^/new W=$w r=$r /" >> $O/summary.txt
  MADRONA_BB_LIB=$V timeout -k 10 200 python tools/ablate.py --worlds $w --iters 200 --rounds 3 --only 0 > $O/old_${w}_${r}.log 2>&1 || exit $?
  grep median $O/old_${w}_${r}.log | sed "s/^/old W=$w r=$r /" >> $O/summary.txt
done
done
timeout -k 10 200 python tools/ablate.py --worlds 8192 --iters 200 --rounds 3 > $O/trace8k_new.log 2>&1 || exit $?
