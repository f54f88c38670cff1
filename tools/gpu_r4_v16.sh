#!/bin/bash
# round 4: headline accumulator copy into LDS read back by inline asm (no compiler vmcnt(0)): parity + A/B
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
V=$PWD/mkfhe_amd/lib/variants
MKFHE_LIB=$V/s2lds5.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "step_kernels" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_lds5_parity.txt 2>&1 || { tail -40 $O/${TAG}_lds5_parity.txt; exit 1; }
tail -1 $O/${TAG}_lds5_parity.txt
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['roofline']['per_launch_us'],2), 'us/launch parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
HL="--steps 3 --warmup 1 --cpu-threads 16"
for rep in 1 2; do
run hl_def$rep "MKACC_STEP=2" "$HL"
run hl_lds5$rep "MKFHE_LIB=$V/s2lds5.so" "$HL"
run hl_lds6$rep "MKFHE_LIB=$V/s2lds6.so" "$HL"
done
