export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/prof1.log 2>&1
rc=$?
cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
exit $rc
