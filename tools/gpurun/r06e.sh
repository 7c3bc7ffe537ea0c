# round 6: which of the round's kernel changes costs rate?  Same-box A/Bs of variant builds of this tree
# (tools/gpurun/_build_variant.sh): base (the tree as is) against relstop (-DSO100_NEWTON_RELSTOP: rounds 3-5's
# relative cost stop instead of the Newton decrement) and nofeat (-DSO100_NO_FEAT: EPA's barycentric witness alone)
export TMPDIR=/tmp
O=gpurun_out/r06e
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
for n in 8192 65536; do
  bash tools/gpurun/ab.sh $O/relstop $V/libso100_hip_base.so $V/libso100_hip_relstop.so $n 3 > $O/ab_relstop_$n.txt 2>&1 || exit $?
  bash tools/gpurun/ab.sh $O/nofeat $V/libso100_hip_base.so $V/libso100_hip_nofeat.so $n 3 > $O/ab_nofeat_$n.txt 2>&1 || exit $?
done
echo R06E_DONE
