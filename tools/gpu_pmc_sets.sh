#!/bin/bash
# usage: gpu_pmc_sets.sh TAG "CTR CTR ..." ["CTR ..."] ...   (one rocprofv3 --pmc pass per set)
# on a shortened bench (n=32 steps per party); summary of the step kernel per set
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
i=0
for CS in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CS -d gpurun_out/pmc_$TAG/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --n-override 32 > gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG
