# round-3 closing set, part 2 (auto mode fused at every size): the bench line at 65,536 (fused, CPU baseline),
# its rocprofv3 kernel trace and per-step PMC traffic, the two full-size tests
export TMPDIR=/tmp
O=gpurun_out/r03close2
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "full_size or step_mode" -v -rA --timeout 300 --timeout-method thread -s > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 60 --warmup 30 --no-cpu-baseline --contact-steps 2 > $O/trace.log 2>&1 || exit $?
B="python bench.py --total-envs 65536 --warmup 40 --steps 5 --no-cpu-baseline --no-kernel-timing --contact-steps 0"
P=$O/pmc_fused_65536
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $P -o fetch --output-format csv -- $B > $P.fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $P -o write --output-format csv -- $B > $P.write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU -d $P -o sq --output-format csv -- $B > $P.sq.log 2>&1 || exit $?
python tools/gpurun/pmc_step_traffic.py $P 65536 fused newton 40 5 $O/r03_pmc_step_fused_newton_65536.json > $P.traffic.log 2>&1 || exit $?
echo R03CLOSE2_DONE
