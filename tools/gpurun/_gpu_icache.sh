# Instruction-fetch diagnosis of the fused vs the split step (writes gpurun_out/icache/*): the SQC
# counter list, then per mode an SQ pass and an SQC instruction-cache pass over a short bench at 65,536 envs.
export TMPDIR=/tmp
O=gpurun_out/icache
rm -rf $O; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -iE "SQC_|ICACHE|INST_CACHE|SQ_IFETCH|SQ_INSTS_|SQ_WAIT" $O/counters.txt | head -80 > $O/counters_sq.txt || true
B="python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-kernel-timing --contact-steps 1"
for mode in 1 0; do
  SO100_FUSED=$mode timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d $O/pmc$mode -o sq --output-format csv -- $B > $O/sq$mode.log 2>&1 || exit $?
  SO100_FUSED=$mode timeout -k 10 -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $O/pmc$mode -o sqc --output-format csv -- $B > $O/sqc$mode.log 2>&1 || echo "sqc pass failed ($mode)" >> $O/notes.txt
done
echo ICDONE
