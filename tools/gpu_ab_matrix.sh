#!/bin/bash
# A/B matrix: tools/gpu_ab_matrix.sh TAG "name|lib.so|ENV=.. ENV2=.." ...
#   each entry: headline EvalAcc bench (its 16-gate oracle check included), ABAB order
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
for rep in 1 2; do
for E in "$@"; do
  IFS='|' read -r n L ENVS <<< "$E"
  env $ENVS MKFHE_LIB=$PWD/$L timeout -k 10 300 python bench.py --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 ${BENCH_ARGS} \
     > gpurun_out/ab_$TAG/$n.$rep.json 2> gpurun_out/ab_$TAG/$n.$rep.err || { echo "$n: bench failed"; tail -5 gpurun_out/ab_$TAG/$n.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$TAG/$n.$rep.json')); print('$n', round(d['value'],1), 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
done
