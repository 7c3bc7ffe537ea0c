# round 5: PGS with 6 or 8 contacts per env held on chip across the sweeps (kResident 4 -> 6 / 8: 206 / 223 VGPRs, no
# scratch, still 2 waves per SIMD) against this tree, 65,536 envs, interleaved; PGS parity subset on the kResident 8 build
export TMPDIR=/tmp
O=gpurun_out/r05v
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
P="python bench.py --solver pgs --no-cpu-baseline --steps 60 --contact-steps 0"
for r in 1 2; do
  timeout -k 10 200 $P > $O/base_$r.json 2> $O/base_$r.err || exit $?
  for k in 6 8; do
    SO100_LIB=$V/libso100_hip_res$k.so timeout -k 10 200 $P > $O/res${k}_$r.json 2> $O/res${k}_$r.err || exit $?
  done
done
SO100_LIB=$V/libso100_hip_res8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pgs and (heavy_contact or step_parity or overflow or pad_contact)" > $O/pytest_res8.log 2>&1 || exit $?
echo R05V_DONE
