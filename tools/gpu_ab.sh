#!/bin/bash
# A/B timing of engine builds: usage gpu_ab.sh TAG LIB.so [LIB.so ...]
# each: GPU parity tests of the accumulator, then the EvalAcc bench (per-launch us)
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
for L in "$@"; do
  n=$(basename $L .so)
  MKFHE_LIB=$PWD/$L timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider ${PARITY_K:+-k "$PARITY_K"} > gpurun_out/ab_$TAG/$n.test 2>&1 || { echo "$n: parity FAILED"; tail -5 gpurun_out/ab_$TAG/$n.test; exit 1; }
  MKFHE_LIB=$PWD/$L timeout -k 10 300 python bench.py --stage evalacc --steps 2 --warmup 1 --cpu-baseline 0 "${BENCH_ARGS[@]}" > gpurun_out/ab_$TAG/$n.json 2> gpurun_out/ab_$TAG/$n.err || { echo "$n: bench failed"; tail -5 gpurun_out/ab_$TAG/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$TAG/$n.json')); print('$n', round(d['value'],1), d['unit'], 'per_launch_us', round(d['roofline']['per_launch_us'],2))"
done
