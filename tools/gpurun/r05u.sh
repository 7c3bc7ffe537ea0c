# round 5: LLVM's AMDGPU register-pressure trackers in the scheduler (-mllvm -amdgpu-use-amdgpu-trackers=1, every
# translation unit; the 3-wave build stays scratch-free), interleaved with this tree at 65,536 and 8,192 envs
export TMPDIR=/tmp
O=gpurun_out/r05u
rm -rf $O; mkdir -p $O
V=gym-so100-c_amd/gym_so100/_lib_var
bash tools/gpurun/ab.sh $O/ab65536 gym-so100-c_amd/gym_so100/_lib/libso100_hip.so $V/libso100_hip_trackers.so 65536 3 > $O/ab65536.txt 2>&1 || exit $?
bash tools/gpurun/ab.sh $O/ab8192 gym-so100-c_amd/gym_so100/_lib/libso100_hip.so $V/libso100_hip_trackers.so 8192 3 > $O/ab8192.txt 2>&1 || exit $?
echo R05U_DONE
