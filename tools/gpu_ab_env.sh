#!/bin/bash
# usage: tools/gpu_ab_env.sh TAG PARAMSET VAR=a VAR=b ...
#   EvalAcc bench under alternative environment settings (e.g. MKACC_DSCR=0
#   MKACC_DSCR=1; one argument may set several variables: "A=1 B=2", and
#   MKFHE_LIB=<path> selects an engine build), ABAB order to expose drift;
#   each run includes the bench's own oracle parity check
TAG=$1; PS=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
for rep in 1 2; do
for E in "$@"; do
  n=$(echo "$E" | sed 's#[^A-Za-z0-9_=.]##g; s#=#_#g' | cut -c1-60)
  env $E timeout -k 10 300 python bench.py --paramset $PS --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 \
     > gpurun_out/ab_$TAG/$n.$rep.json 2> gpurun_out/ab_$TAG/$n.$rep.err || { echo "$n: bench failed"; tail -5 gpurun_out/ab_$TAG/$n.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$TAG/$n.$rep.json')); print('$PS $E', round(d['value'],1), 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
done
