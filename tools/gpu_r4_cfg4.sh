#!/bin/bash
# round 4: config 4 (STD128_MKNTRU_3, k=8, dg=4) -- mk_step_kernel + d_i scratch (MKACC_STEP=1)
# against mk_step2_kernel at one wave per SIMD (MKACC_STEP=2), full gates at B=8192, ABAB
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
for rep in 1 2; do
for V in 1 2; do
  MKACC_STEP=$V timeout -k 10 300 python bench.py --paramset STD128_MKNTRU_3 --batch 8192 --steps 1 --warmup 1 --cpu-threads 16 \
     > $O/${TAG}_c4_v$V.$rep.json 2> $O/${TAG}_c4_v$V.$rep.err || { echo "c4 v$V failed"; tail -5 $O/${TAG}_c4_v$V.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_c4_v$V.$rep.json')); print('c4 v$V', round(d['value'],1), 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
done
