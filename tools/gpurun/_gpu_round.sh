# round-end measurement set (writes gpurun_out/r01/*): parity tests, smoke, bench line (default solver:
# Newton), kernel trace, PMC traffic of the solver kernel, SQ counters; then the PGS bench line and trace.
export TMPDIR=/tmp
O=gpurun_out/r01
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
B="python bench.py --steps 4 --warmup 60 --no-cpu-baseline --no-kernel-timing --contact-steps 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o fetch --output-format csv -- $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc -o write --output-format csv -- $B > $O/pmc_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc -o sq --output-format csv -- $B > $O/pmc_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc -o misc --output-format csv -- $B > $O/pmc_misc.log 2>&1 || exit $?
python tools/gpurun/_pmc_traffic.py $O/pmc 16384 $O/pmc_traffic_newton.json 4 newton > $O/pmc_traffic.log 2>&1 || exit $?
python tools/gpurun/_pmc_report.py $O/pmc > $O/pmc_report.txt 2>&1 || exit $?
python tools/gpurun/_trace_report.py $O/trace > $O/trace_report.txt 2>&1 || exit $?
lscpu > $O/lscpu.txt 2>&1; nproc > $O/nproc.txt; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS" >> $O/nproc.txt
timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline > $O/bench_pgs.json 2> $O/bench_pgs.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_pgs -o bench_pgs --output-format csv -- python bench.py --solver pgs --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace_pgs.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dev/render_bench.py $O/render_bench.json > $O/render_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_render -o render --output-format csv -- python tools/dev/render_bench.py $O/render_bench_prof.json > $O/trace_render.log 2>&1 || exit $?
echo ROUNDDONE
