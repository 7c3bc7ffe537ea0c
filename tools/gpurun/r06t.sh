# round 6: the convex collider's phase cycles (GJK / EPA and inside EPA) at 8,192 and 65,536 envs, fused step
# (-DSO100_EPA_STAMPS variant, tools/dev/epa_stamps.py)
export TMPDIR=/tmp
O=gpurun_out/r06t
rm -rf $O; mkdir -p $O
for n in 8192 65536; do
  SO100_LIB=gym-so100-c_amd/gym_so100/_lib_var/libso100_hip_epastamps.so timeout -k 10 200 python tools/dev/epa_stamps.py $n fused >> $O/epa_stamps.txt 2>&1 || exit $?
done
cat $O/epa_stamps.txt
