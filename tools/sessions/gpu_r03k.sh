set -u
O=gpurun_out/r03k; mkdir -p $O
for r in 1 2; do
for w in 8192 16384 32768; do
  timeout -k 10 200 python tools/ablate.py --worlds $w --iters 200 --rounds 3 --only 0 > $O/base_${w}_$r.log 2>&1 || exit $?
  grep median $O/base_${w}_$r.log | sed "s/^/base W=$w r=$r /" >> $O/summary.txt
  for a in 2 16 17 18; do
    MADRONA_BB_LIB=$PWD/madrona_basketball_amd/_variants/aux$a/libmadrona_basketball_amd.so timeout -k 10 200 python tools/ablate.py --worlds $w --iters 200 --rounds 3 --only 0 > $O/aux${a}_${w}_$r.log 2>&1 || exit $?
    grep median $O/aux${a}_${w}_$r.log | sed "s/^/aux$a W=$w r=$r /" >> $O/summary.txt
  done
done
done
