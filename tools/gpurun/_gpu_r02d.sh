# fused kernel: chunk count and shard size sweep, and its instruction-cache counters (gpurun_out/r02d/*)
export TMPDIR=/tmp
O=gpurun_out/r02d
rm -rf $O; mkdir -p $O
for n in 65536 32768 16384 8192; do
  B="python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10"
  for c in 1 2 4; do SO100_CHUNKS=$c timeout -k 10 200 $B > $O/fused_c${c}_$n.json 2>$O/err || exit $?; done
  SO100_FUSED=0 timeout -k 10 200 $B > $O/split_$n.json 2>$O/err || exit $?
done
B="python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-kernel-timing --contact-steps 1"
for mode in 1 0; do
  SO100_FUSED=$mode timeout -k 10 -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $O/pmc$mode -o sqc --output-format csv -- $B > $O/sqc$mode.log 2>&1 || exit $?
  SO100_FUSED=$mode timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d $O/pmc$mode -o sq --output-format csv -- $B > $O/sq$mode.log 2>&1 || exit $?
done
python tools/gpurun/_pmc_sum.py $O/pmc1 $O/pmc0 > $O/pmc_sum.txt 2>&1
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f); done
echo R02DDONE
