#!/bin/bash
# round 4: config 4 with the d_i reloads in d_i reload prefetch distance 3 and 1 (MKACC_DSCR_PF) vs the default 2
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['per_launch_us'],2), 'us/step', d['roofline']['kernel'], 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C4="--stage evalacc --steps 1 --warmup 1 --paramset STD128_MKNTRU_3 --batch 8192"
V=$PWD/mkfhe_amd/lib/variants
run c4_base "" "$C4"
run c4_pf3 "MKFHE_LIB=$V/pf3.so" "$C4"
run c4_pf1 "MKFHE_LIB=$V/pf1.so" "$C4"
run c4_base2 "" "$C4"
run c4_pf3b "MKFHE_LIB=$V/pf3.so" "$C4"
