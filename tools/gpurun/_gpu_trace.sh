export TMPDIR=/tmp
O=gpurun_out/t
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o bench --output-format csv -- python bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
echo TDONE
