# pad-contact parity tests (no -x) and a bench A/B against the no-pads variant (writes gpurun_out/pads/*)
export TMPDIR=/tmp
O=gpurun_out/pads
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rA -s --timeout 120 --timeout-method thread -k "pad or hull_table or mpr or self_collision or random" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpurun/_gpu_ab.sh nopads > $O/ab.log 2>&1 || exit $?
echo PDONE
