# stage phase stamps on the final round-3 kernels (split stage kernel, the box-box pairs alone in the "Euler" slot)
export TMPDIR=/tmp
O=gpurun_out/r03dd
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for n in 8192 65536; do
  SO100_FUSED=0 SO100_LIB=$V/libso100_hip_sstamps_final.so timeout -k 10 200 python tools/gpurun/_stage_stamps_report.py newton $n > $O/sstamps_$n.txt 2>&1 || exit $?
done
echo R03DD_DONE
