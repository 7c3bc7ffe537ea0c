# round 6: the Base-fold parity class (test_base_contact_parity, Newton) under the Newton stop variants: cur (gradient
# noise stop at 16 float epsilons of the terms), k8 (8), k0 (off: the decrement alone), prev (16, the scanned top-face /
# snap vertex); plus the deep-fold siblings (self-collision, pad-link) on cur and k8
export TMPDIR=/tmp
O=gpurun_out/r06i
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
T="python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread -rf"
for v in cur k8 k0 prev; do
  L=""; [ $v = k8 ] && L=$V/libso100_hip_k8.so; [ $v = k0 ] && L=$V/libso100_hip_k0.so; [ $v = prev ] && L=$V/libso100_hip_base.so
  SO100_LIB=$L timeout -k 10 600 $T -k "test_base_contact_parity and newton" > $O/base_$v.log 2>&1; rc=$?
  if [ $rc -gt 1 ]; then exit $rc; fi
done
for v in cur k8; do
  L=""; [ $v = k8 ] && L=$V/libso100_hip_k8.so
  SO100_LIB=$L timeout -k 10 900 $T -k "(test_self_collision_parity or test_pad_link_contact_parity or test_overflow_contact_parity) and newton" > $O/deep_$v.log 2>&1; rc=$?
  if [ $rc -gt 1 ]; then exit $rc; fi
done
for f in $O/*.log; do echo "== $f"; grep -E "ensemble floor|passed|failed" $f; done
echo R06I_DONE
