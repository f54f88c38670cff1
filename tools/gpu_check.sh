#!/bin/bash
# usage: tools/gpu_check.sh TAG
#   parity first (primitives + EvalAcc), then the whole -m gpu suite, then a
#   short headline bench and its rocprof kernel summary; stops at the first failure
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/parity_$TAG.txt 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/parity_$TAG.txt; exit 1; }
tail -2 gpurun_out/parity_$TAG.txt
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v ${PYTEST_EXTRA} --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_$TAG.txt 2>&1 || { echo "suite FAILED"; tail -30 gpurun_out/pytest_$TAG.txt; exit 1; }
tail -2 gpurun_out/pytest_$TAG.txt
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench FAILED"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(round(d['value'],1), d['unit'], 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof FAILED"; exit 1; }
echo done
