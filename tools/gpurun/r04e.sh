# round 4: overflow outliers in detail (pre-marker tree abtree/cur) and its overflow-path A/B; the separating-direction
# cache A/B; the marker / overflow / bitwise GPU tests on this tree
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04e
rm -rf $O; mkdir -p $O
L=gym-so100-c_amd/gym_so100/_lib_var
# the cache must not change a single bit: 8,192 envs x 100 random-action steps through both libraries
for v in nosep sep; do
  SO100_LIB=$L/libso100_hip_$v.so timeout -k 10 200 python tools/dev/lib_states.py 8192 100 $O/st_$v.npz > $O/st_$v.log 2>&1 || exit $?
done
python - $O > $O/st_compare.txt 2>&1 <<'PY' || exit $?
import sys, numpy as np
o = sys.argv[1]
a, b = np.load(f"{o}/st_nosep.npz"), np.load(f"{o}/st_sep.npz")
for k in a.files:
    print(k, "bitwise equal" if np.array_equal(a[k], b[k]) else f"DIFFER max {np.abs(a[k].astype(float) - b[k].astype(float)).max():.3e}")
PY
bash tools/gpurun/ab.sh $O/ab_sep $L/libso100_hip_nosep.so $L/libso100_hip_sep.so 65536 3 > $O/ab_sep_65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab_sep $L/libso100_hip_nosep.so $L/libso100_hip_sep.so 8192 3 > $O/ab_sep_8192.txt 2>&1 || exit $?
(cd abtree/cur && timeout -k 10 300 python -u tools/dev/overflow_outliers.py newton 1 > $O/outliers_newton1.log 2>&1) || exit $?
(cd abtree/cur && bash tools/gpurun/ab.sh $O/ab_noovf $L/libso100_hip_head.so $L/libso100_hip_noovf.so 65536 3 > $O/ab_noovf_65536.txt 2>&1) || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "ee_weld or chunking or fused_step_matches or product_builds or overflow" > $O/tests.log 2>&1; echo "pytest rc=$?" >> $O/tests.log
echo R04E_DONE
