#!/bin/bash
# round 4: config 4 on the final build with 2, 4 and 3 batch slices (MKACC_STREAMS)
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['per_launch_us'],2), 'us/step', d['roofline']['kernel'], 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
C4="--stage evalacc --steps 1 --warmup 1 --paramset STD128_MKNTRU_3 --batch 8192"
run c4_s2 "MKACC_STREAMS=2" "$C4"
run c4_s4 "MKACC_STREAMS=4" "$C4"
run c4_s3 "MKACC_STREAMS=3" "$C4"
run c4_s2b "MKACC_STREAMS=2" "$C4"
run c4_s4b "MKACC_STREAMS=4" "$C4"
