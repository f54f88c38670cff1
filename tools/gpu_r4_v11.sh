#!/bin/bash
# round 4: mk_step3_kernel at 3 / 4 waves per SIMD (2-slot key groups): headline and config 4
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C4="--stage evalacc --steps 1 --warmup 1 --cpu-threads 16 --paramset STD128_MKNTRU_3 --batch 8192"
HL="--steps 3 --warmup 1 --cpu-threads 16"
V=$PWD/mkfhe_amd/lib/variants
run hl_w3g2 "MKACC_STEP=3 MKFHE_LIB=$V/s3w3g2.so" "$HL"
run hl_w4g2 "MKACC_STEP=3 MKFHE_LIB=$V/s3w4g2.so" "$HL"
run c4_w3g2 "MKACC_STEP=3 MKFHE_LIB=$V/s3w3g2.so" "$C4"
run hl_s2 "MKACC_STEP=2" "$HL"
