# graph replay vs eager launches of the env step at the strong-scaling shard sizes (gpurun_out/g/*)
export TMPDIR=/tmp
O=gpurun_out/g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "graph or teacher_forced or goal_env" > $O/pytest.log 2>&1 || exit $?
for n in 8192 16384 65536; do
  for gr in 0 1; do
    SO100_GRAPH=$gr timeout -k 10 200 python bench.py --no-cpu-baseline --no-kernel-timing --total-envs $n --steps 200 --warmup 20 > $O/bench_${n}_g$gr.json 2>$O/bench_${n}_g$gr.err || exit $?
  done
done
echo GDONE
