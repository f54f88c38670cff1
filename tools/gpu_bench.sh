#!/bin/bash
# usage: PROF=1 tools/gpu_bench.sh TAG [extra bench args]
#   parity tests + smoke + bench (+ rocprofv3 kernel stats when PROF=1)
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/smoke_$TAG.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
[ $rc -ne 0 ] && exit $rc
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 "$@" > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; head -4 gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -c1-200
fi
exit $rc
