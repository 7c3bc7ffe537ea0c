# round 6: the Base-fold parity class (test_base_contact_parity[newton]) and the bitwise build tests on three libraries:
# cur (the move uncontracted, __fmul_rn / __fadd_rn, + no cost after a quadratic-exact stop); earlier: explicit FMAs and
# the move as written (skipnofma), both the same results, which differ from
# prev (before both)
export TMPDIR=/tmp
O=gpurun_out/r06w
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_order.py -v -s --timeout 300 --timeout-method thread -rf"
for v in cur prev; do
  L=""; [ $v != cur ] && L=$V/libso100_hip_$v.so
  SO100_LIB=$L timeout -k 10 600 $T -k "test_base_contact_parity or pool_contention or order or fused_step_matches" > $O/$v.log 2>&1; rc=$?
  echo "$v rc $rc: $(tail -1 $O/$v.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
for v in cur prev; do echo "== $v"; grep -E "\[newton Base|\[Base|Base\]" $O/$v.log | head -3; done
echo R06W_DONE
