#!/bin/bash
# round 4: bench with the cpu-seconds baseline sample (headline, config 4)
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 400 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -20 $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
timeout -k 10 400 python bench.py --stage evalacc --steps 1 --warmup 1 --paramset STD128_MKNTRU_3 --batch 8192 \
   > $O/${TAG}_c4.json 2> $O/${TAG}_c4.err || { tail -5 $O/${TAG}_c4.err; exit 1; }
cat $O/${TAG}_c4.json
