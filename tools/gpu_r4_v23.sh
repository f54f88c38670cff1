#!/bin/bash
# round 4: config-4 cache-policy A/B of mk_step_kernel's accumulator and d_i scratch accesses
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['per_launch_us'],2), 'us/step', d['roofline']['kernel'], 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C4="--stage evalacc --steps 1 --warmup 1 --cpu-threads 16 --paramset STD128_MKNTRU_3 --batch 8192"
V=$PWD/mkfhe_amd/lib/variants
run c4_base "MKACC_STEP=1" "$C4"
run c4_accnt "MKFHE_LIB=$V/accnt.so" "$C4"
run c4_accnt_dsnt "MKFHE_LIB=$V/accnt_dsnt.so" "$C4"
run c4_dsnt "MKFHE_LIB=$V/dsnt.so" "$C4"
run c4_base2 "MKACC_STEP=1" "$C4"
run c4_accnt2 "MKFHE_LIB=$V/accnt.so" "$C4"
