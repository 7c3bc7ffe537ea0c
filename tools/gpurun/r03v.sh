# round-3 pass V: hardware reciprocals in the Newton setup, Euler rsq normalisation, box-box clipping and collision reciprocals (A/B vs HEAD); fused 2- vs
# 3-wave build and the split step at the 2- and 4-GPU shard sizes
export TMPDIR=/tmp
O=gpurun_out/r03v
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpurun/ab.sh $O/a $V/libso100_hip_base.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 8192 3 > $O/ab_8192.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/b $V/libso100_hip_base.so gym-so100-c_amd/gym_so100/_lib/libso100_hip.so 65536 2 > $O/ab_65536.txt 2>&1 || exit $?
for n in 16384 32768; do
  for mode in w2 w3 split; do
    case $mode in w2) E="SO100_FUSED_WAVES=2";; w3) E="SO100_FUSED_WAVES=3";; split) E="SO100_FUSED=0";; esac
    env $E timeout -k 10 200 python bench.py --total-envs $n --no-cpu-baseline --steps 200 --contact-steps 0 > $O/bench_${n}_$mode.json 2> $O/bench_${n}_$mode.err || exit $?
  done
done
grep -E "passed|failed" $O/pytest_gpu.log | tail -1
cat $O/ab_*.txt
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e6,3), d['config']['step_mode'], d['config']['fused_build'])"; done
