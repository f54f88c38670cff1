#!/bin/bash
# round 4: headline accumulator copy into LDS (MKACC_S2_NXPF=1) A/B, widereg2 scheduler / prefetch A/B
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
HL="--steps 3 --warmup 1 --cpu-threads 16"
C5="--paramset STD100_MKNTRU --q-bits 50 --stage evalacc --steps 2 --warmup 1 --cpu-threads 16"
V=$PWD/mkfhe_amd/lib/variants
for rep in 1 2; do
run hl_def$rep "MKACC_STEP=2" "$HL"
run hl_lds5$rep "MKFHE_LIB=$V/s2lds5.so" "$HL"
run hl_lds3$rep "MKFHE_LIB=$V/s2lds3.so" "$HL"
done
for rep in 1 2; do
run c5_def$rep "MKACC_WREG2=1" "$C5"
run c5_mmc$rep "MKFHE_LIB=$V/w2mmc.so" "$C5"
run c5_pf2$rep "MKFHE_LIB=$V/w2pf2.so" "$C5"
done
