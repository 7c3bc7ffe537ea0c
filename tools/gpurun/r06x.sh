# round 6 dev probe: the state after each of 20 steps (4,096 envs) under the Newton move's arithmetic (fma: explicit
# FMAs, unc: __fmul_rn / __fadd_rn, wr: as written) with (1) and without (0, compiled, never taken) the skipped cost
# after a quadratic-exact stop, against prev (the tree before both) and cur (unc, skip): which ones change results?
export TMPDIR=/tmp
O=gpurun_out/r06x
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
timeout -k 10 120 python tools/dev/lib_states_ab.py $O/cur.npz 4096 20 || exit $?
for v in prev fma1 fma0 unc0 wr1 wr0; do
  SO100_LIB=$V/libso100_hip_$v.so timeout -k 10 120 python tools/dev/lib_states_ab.py $O/$v.npz 4096 20 || exit $?
done
python - $O <<'PY'
import numpy as np, sys
o = sys.argv[1]
names = ("prev", "wr0", "wr1", "fma0", "fma1", "unc0", "cur")
L = {k: np.load(f"{o}/{k}.npz")["q"] for k in names}
for a in names:
    print(a, " ".join(f"{b}:{int((L[a] != L[b]).any(axis=2).any(axis=0).sum())}" for b in names))
PY
