# env-range chunking A/B (SO100_CHUNKS) at the bench's sizes (writes gpurun_out/c/*)
export TMPDIR=/tmp
O=gpurun_out/c
rm -rf $O; mkdir -p $O
for n in 65536 8192; do
  for k in 4 5 6 8 4; do
    SO100_CHUNKS=$k timeout -k 10 200 python bench.py --no-cpu-baseline --no-kernel-timing --total-envs $n --steps 150 --warmup 20 > $O/b_${n}_$k.json 2>$O/b_${n}_$k.err || exit $?
    echo $n $k $(grep -o '"value": [0-9.]*' $O/b_${n}_$k.json) >> $O/summary.txt
  done
done
echo CDONE
