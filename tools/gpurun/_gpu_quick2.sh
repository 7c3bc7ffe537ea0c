# quick check: fused/step-mode/chunking parity tests + bench at 65,536 and 8,192 envs (gpurun_out/q2/*)
export TMPDIR=/tmp
O=gpurun_out/q2
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "fused or step_mode or chunking or graph or smoke or heavy or pad or mpr" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for n in 65536 8192; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --total-envs $n --steps 100 --warmup 10 > $O/b_$n.json 2>$O/err || exit $?
done
B="python bench.py --steps 4 --warmup 30 --no-cpu-baseline --no-kernel-timing --contact-steps 1"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc -o write --output-format csv -- $B > $O/pmc_write.log 2>&1 || exit $?
python tools/gpurun/_pmc_report.py $O/pmc | grep -A2 write
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*' $f); done
