# round 6, VERDICT r5 item 2: the driver's bench window (--steps 20 --warmup 5) against the builder's (300 / 30).
# (1) per-step device time from reset of round 4's tree (77bb484), round 5's closing tree (f9234e6) and this tree;
# (2) the driver's exact command on round 4's and round 5's trees, interleaved, 3 runs each;
# (3) 20-step windows after 5, 30 and 300 warmup steps on this tree.
export TMPDIR=/tmp
O=gpurun_out/r06a
rm -rf $O; mkdir -p $O
# the round-6 pool (sized to the resident waves) first: bitwise builds, none_free == 0, the 65,536-env footprint
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 240 --timeout-method thread \
  -k "pool or contact_record_memory" > $O/pytest_pool.log 2>&1 || exit $?
for t in r04 r05 cur; do
  R=abtree/$t; [ $t = cur ] && R=.
  timeout -k 10 200 python tools/gpurun/step_series.py $R 65536 400 $O/series_$t.json > $O/series_$t.txt 2>&1 || exit $?
done
for r in 1 2 3; do
  for t in r04 r05; do
    (cd abtree/$t && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline) > $O/drv_${t}_$r.json 2> $O/drv_${t}_$r.err || exit $?
  done
done
for w in 5 30 300; do
  for r in 1 2; do
    timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-cpu-baseline > $O/win_w${w}_$r.json 2> $O/win_w${w}_$r.err || exit $?
  done
done
for t in r04 r05 cur; do
  R=abtree/$t; [ $t = cur ] && R=.
  timeout -k 10 200 python tools/gpurun/step_series.py $R 65536 400 $O/series2_$t.json > $O/series2_$t.txt 2>&1 || exit $?
done
echo R06A_DONE
