# box-box SAT: all 15 axes first, one separation test, then the serial selection (sat) vs HEAD (head): bitwise state equality after
# 40 steps at 8,192 (2-wave build) and 16,384 envs (3-wave), GPU suite on sat, A/B
export TMPDIR=/tmp
O=gpurun_out/r03ff
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for n in 8192 16384; do
  for v in head sat; do
    SO100_LIB=$V/libso100_hip_$v.so timeout -k 10 200 python tools/dev/lib_states.py $n 40 $O/st_${v}_$n.npz >> $O/states.log 2>&1 || exit $?
  done
done
python - $O >> $O/states.log 2>&1 <<'PY' || exit $?
import sys, numpy as np
o = sys.argv[1]
for n in (8192, 16384):
    a, b = np.load(f"{o}/st_head_{n}.npz"), np.load(f"{o}/st_sat_{n}.npz")
    print(n, {k: bool(np.array_equal(a[k], b[k])) for k in a.files})
PY
SO100_LIB=$V/libso100_hip_sat.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu_sat.log 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/rne65536 $V/libso100_hip_head.so $V/libso100_hip_sat.so 65536 3 > $O/ab_sat_65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/rne8192 $V/libso100_hip_head.so $V/libso100_hip_sat.so 8192 3 > $O/ab_sat_8192.txt 2>&1 || exit $?
echo R03FF_DONE
