# arm-contact qvel error, GPU vs the fp32 oracle floor, in-tree build vs a variant (tools/dev/padlink_err.py)
export TMPDIR=/tmp
V=gym-so100-c_amd/gym_so100/_lib_var
for s in pgs newton; do
  echo "== base $s"; timeout -k 10 300 python tools/dev/padlink_err.py 384 $s 2>&1 | grep -v amdgpu.ids || exit $?
  echo "== $1 $s"; SO100_LIB=$V/libso100_hip_$1.so timeout -k 10 300 python tools/dev/padlink_err.py 384 $s 2>&1 | grep -v amdgpu.ids || exit $?
done
