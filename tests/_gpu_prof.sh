export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
B="python bench.py --steps 6 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc -o sq --output-format csv -- $B > gpurun_out/pmc/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch --output-format csv -- $B > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc -o write --output-format csv -- $B > gpurun_out/pmc/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/pmc -o misc --output-format csv -- $B > gpurun_out/pmc/misc.log 2>&1 || exit $?
echo PROFDONE
