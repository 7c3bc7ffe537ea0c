# round 5: the GPU suite on per-wave pool entries; a same-box A/B of the PGS env order (SO100_PGS_ORDER=0: round 4's
# dispatch) with rocprofv3 kernel stats of both (the order kernel's share); bench lines at 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05d
rm -rf $O; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rA --timeout 400 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for r in 1 2; do
  SO100_PGS_ORDER=0 timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline --steps 100 --contact-steps 0 > $O/pgs_noorder_$r.json 2> $O/pgs_noorder_$r.err || exit $?
  timeout -k 10 300 python bench.py --solver pgs --no-cpu-baseline --steps 100 --contact-steps 0 > $O/pgs_order_$r.json 2> $O/pgs_order_$r.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_pgs_order -o pgs --output-format csv -- python bench.py --solver pgs --steps 20 --warmup 10 --no-cpu-baseline --contact-steps 0 > $O/trace_pgs_order.log 2>&1 || exit $?
SO100_PGS_ORDER=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_pgs_noorder -o pgs --output-format csv -- python bench.py --solver pgs --steps 20 --warmup 10 --no-cpu-baseline --contact-steps 0 > $O/trace_pgs_noorder.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --total-envs 8192 --no-cpu-baseline > $O/bench_8192.json 2> $O/bench_8192.err || exit $?
echo R05D_DONE
