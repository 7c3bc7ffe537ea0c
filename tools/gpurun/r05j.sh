# round 5: instruction-fetch and issue-stall counters of the fused step at 65,536 envs (separate passes)
export TMPDIR=/tmp
O=gpurun_out/r05j
rm -rf $O; mkdir -p $O
B="python bench.py --total-envs 65536 --warmup 10 --steps 3 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $O/ic -o ic --output-format csv -- $B > $O/ic.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o sq --output-format csv -- $B > $O/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM -d $O/sq2 -o sq2 --output-format csv -- $B > $O/sq2.log 2>&1 || exit $?
echo R05J_DONE
