# per-GPU rate at the shard sizes the 8-GPU strong-scaling run uses (writes gpurun_out/s/*)
export TMPDIR=/tmp
O=gpurun_out/s
mkdir -p $O
for n in 8192 16384 32768 65536; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 200 --warmup 20 > $O/bench_$n.json 2>$O/bench_$n.err || exit $?
done
for n in 8192 65536; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$n -o t --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --total-envs $n > $O/trace_$n.log 2>&1 || exit $?
done
echo SDONE
