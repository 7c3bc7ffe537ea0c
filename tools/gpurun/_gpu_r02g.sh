# fused (debug-free instantiation) vs split per shard size, twice, same box (gpurun_out/r02g/*)
export TMPDIR=/tmp
O=gpurun_out/r02g
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fused or step_mode or graph" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for n in 65536 49152 32768; do for f in 1 0; do
  SO100_FUSED=$f timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/f${f}_${n}_$i.json 2>$O/err || exit $?
done; done; done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f); done
