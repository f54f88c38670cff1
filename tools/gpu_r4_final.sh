#!/bin/bash
# round 4 final validation: GPU suite, smoke, headline bench + kernel stats, config 5 and config 4 bench + kernel stats
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
TAG=$TAG bash tools/gpu_r4_base.sh || exit 1
timeout -k 10 300 python bench.py --paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 \
   > $O/${TAG}_c5.json 2> $O/${TAG}_c5.err || { tail -5 $O/${TAG}_c5.err; exit 1; }
cat $O/${TAG}_c5.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_c5prof -o run --output-format csv -- python3 bench.py --paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 1 --warmup 1 --cpu-baseline 0 > $O/${TAG}_c5prof.log 2>&1 || { tail -20 $O/${TAG}_c5prof.log; exit 1; }
find $O/${TAG}_c5prof -name "*kernel_stats.csv" | head -1 | xargs head -3 | cut -c1-200
timeout -k 10 400 python bench.py --stage evalacc --steps 1 --warmup 1 --cpu-threads 16 --paramset STD128_MKNTRU_3 --batch 8192 \
   > $O/${TAG}_c4.json 2> $O/${TAG}_c4.err || { tail -5 $O/${TAG}_c4.err; exit 1; }
cat $O/${TAG}_c4.json
