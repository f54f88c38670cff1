#!/bin/bash
# usage: tools/gpu_ab_cfg5.sh TAG "ENV..." ...
#   config-5 stress (STD100_MKNTRU shape, 50-bit Q, B_g = 2^10) EvalAcc bench under
#   alternative settings (MKACC_WIDE_FP=0/1, MKFHE_LIB=<variant>), ABAB order;
#   every run includes the bench's 16-gate oracle check
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
for rep in 1 2; do
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python bench.py --paramset STD100_MKNTRU --q-bits 50 --steps 1 --warmup 1 --cpu-threads 16 \
     > gpurun_out/ab_$TAG/v$i.$rep.json 2> gpurun_out/ab_$TAG/v$i.$rep.err || { echo "v$i: bench failed"; tail -5 gpurun_out/ab_$TAG/v$i.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$TAG/v$i.$rep.json')); print('$E'.split('/')[-1], round(d['value'],1), 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
done
