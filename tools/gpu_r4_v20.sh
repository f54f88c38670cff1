#!/bin/bash
# round 4: batch slices on two streams by default -- GPU suite, smoke, headline bench + kernel stats,
# config 5 slices A/B + kernel stats, config 4
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
TAG=$TAG bash tools/gpu_r4_base.sh || exit 1
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['per_launch_us'],2), 'us/step slices', d['roofline'].get('slices_per_step'), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C5="--paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16"
for rep in 1 2; do
run c5_s1.$rep "MKACC_STREAMS=1" "$C5"
run c5_s2.$rep "MKACC_STREAMS=2" "$C5"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_c5prof -o run --output-format csv -- python3 bench.py --paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 1 --warmup 1 --cpu-baseline 0 > $O/${TAG}_c5prof.log 2>&1 || { tail -20 $O/${TAG}_c5prof.log; exit 1; }
find $O/${TAG}_c5prof -name "*kernel_stats.csv" | head -1 | xargs head -3 | cut -c1-200
run c4 "" "--stage evalacc --steps 1 --warmup 1 --cpu-threads 16 --paramset STD128_MKNTRU_3 --batch 8192"
