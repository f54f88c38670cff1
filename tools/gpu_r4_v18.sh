#!/bin/bash
# round 4: two-stream half batches (MKACC_STREAMS=2): parity, then headline and config-4 A/B
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "two_stream" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_streams_parity.txt 2>&1 || { tail -40 $O/${TAG}_streams_parity.txt; exit 1; }
tail -1 $O/${TAG}_streams_parity.txt
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['roofline']['per_launch_us'],2), 'us/launch', round(d['ms_per_step'],2), 'ms/step parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
HL="--steps 3 --warmup 1 --cpu-threads 16"
C4="--stage evalacc --steps 1 --warmup 1 --cpu-threads 16 --paramset STD128_MKNTRU_3 --batch 8192"
for rep in 1 2; do
run hl_s1$rep "MKACC_STREAMS=1" "$HL"
run hl_s2$rep "MKACC_STREAMS=2" "$HL"
done
run c4_s1 "MKACC_STREAMS=1" "$C4"
run c4_s2 "MKACC_STREAMS=2" "$C4"
