# per-GPU rate at the strong-scaling shard sizes, and the chunk count at the small shards (gpurun_out/s2/*)
export TMPDIR=/tmp
O=gpurun_out/s2
mkdir -p $O
for n in 8192 16384 32768 65536; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 200 --warmup 20 > $O/bench_$n.json 2>$O/bench_$n.err || exit $?
done
for k in 1 2; do
  for n in 8192 16384; do
    SO100_CHUNKS=$k timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 200 --warmup 20 > $O/bench_${n}_c$k.json 2>$O/bench_${n}_c$k.err || exit $?
  done
done
echo SDONE
