# round 6: which round-5 change made the 65,536-env step slower?  Per-step device time from reset
# (tools/gpurun/step_series.py, 400 steps) of each round-5 milestone tree, two interleaved passes on one box:
# r04 77bb484, f2 6eb9309 (exact table edges), nospill 1804094, pool 77347e0, counts dab4a83, xcd 4372fd4,
# w2tu 164871c, r05 f9234e6, cur (this tree)
export TMPDIR=/tmp
O=gpurun_out/r06b
rm -rf $O; mkdir -p $O
for pass in 1 2; do
  for t in r04 f2 nospill pool counts xcd w2tu r05 cur; do
    R=abtree/$t; [ $t = cur ] && R=.
    timeout -k 10 200 python tools/gpurun/step_series.py $R 65536 400 $O/s${pass}_$t.json > $O/s${pass}_$t.txt 2>&1 || exit $?
  done
done
echo R06B_DONE
