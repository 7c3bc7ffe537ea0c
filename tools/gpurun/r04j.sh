# round 4: the base deep-fold outlier (state 98) substep by substep, GPU vs fp64 / fp32 / fp32-FMA
export TMPDIR=/tmp
O=gpurun_out/r04j
rm -rf $O; mkdir -p $O
timeout -k 10 200 python -u tools/dev/substep_trace.py tools/dev/_states_base.npz s98 newton 10 > $O/trace_s98.log 2>&1 || exit $?

echo R04J_DONE
