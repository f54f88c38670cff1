#!/bin/bash
# usage: tools/gpu_pcsamp.sh TAG [LIB.so]  -- stochastic PC sampling of a short headline run
TAG=$1; LIB=${2:-}
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$LIB" ] && export MKFHE_LIB=$PWD/$LIB
rocprofv3 -L > gpurun_out/pcs_avail_$TAG.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 65536 -d gpurun_out/pcs_$TAG -o run --output-format csv -- \
  python3 bench.py --stage evalacc --steps 1 --warmup 0 --cpu-baseline 0 --n-override 32 > gpurun_out/pcs_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pcs_$TAG.log
find gpurun_out/pcs_$TAG -name "*.csv" | head
exit $rc
