#!/bin/bash
# round 4: config-4 mk_step_kernel (dg = 4, d_i scratch) scheduler / scratch-prefetch A/B
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C4="--stage evalacc --steps 1 --warmup 1 --cpu-threads 16 --paramset STD128_MKNTRU_3 --batch 8192"
V=$PWD/mkfhe_amd/lib/variants
for rep in 1 2; do
run c4_def$rep "MKACC_STEP=1" "$C4"
run c4_mmc$rep "MKFHE_LIB=$V/c4mmc.so" "$C4"
run c4_mmcpf3$rep "MKFHE_LIB=$V/c4mmcpf3.so" "$C4"
done
