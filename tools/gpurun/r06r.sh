# round 6: issue-stall and instruction-mix counters of the fused step on the closing kernels, 65,536 and 8,192 envs
# (separate rocprofv3 --pmc passes, bench.py --warmup 10 --steps 3: 13 fused launches each), summarised by
# tools/gpurun/_sq_report.py
export TMPDIR=/tmp
O=gpurun_out/r06r
rm -rf $O; mkdir -p $O
for n in 65536 8192; do
  B="python bench.py --total-envs $n --warmup 10 --steps 3 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq_$n -o sq --output-format csv -- $B > $O/sq_$n.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM -d $O/sq2_$n -o sq2 --output-format csv -- $B > $O/sq2_$n.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $O/sq3_$n -o sq3 --output-format csv -- $B > $O/sq3_$n.log 2>&1 || exit $?
  python tools/gpurun/_sq_report.py $O $n > $O/sq_report_$n.txt 2>&1 || exit $?
done
cat $O/sq_report_*.txt
echo R06R_DONE
