# round 4: the CRBA / RNE sums as DPP tree scans in every build (this tree) -- the whole GPU suite (bitwise
# builds, the ensemble-gated parity tests), then a same-box A/B against the serial-order build (_lib_var/base)
export TMPDIR=/tmp
O=gpurun_out/r04l
rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
V=gym-so100-c_amd/gym_so100/_lib_var; T=gym-so100-c_amd/gym_so100/_lib/libso100_hip.so
bash tools/gpurun/ab.sh $O/ab8192 $V/libso100_hip_base.so $T 8192 3 > $O/ab8192.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab65536 $V/libso100_hip_base.so $T 65536 3 > $O/ab65536.txt 2>&1 || exit $?
cat $O/ab8192.txt $O/ab65536.txt
echo R04L_DONE
