#!/bin/bash
# round 4: config-4 halves with sc1 read-backs (default 2-slot groups and 4-slot groups, full-size parity in the bench),
# then the config-5 widereg A/B and PMC
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
for E in "h22|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_STEP=2" "h40|mkfhe_amd/lib/variants/h40.so|MKACC_STEP=2"; do
  IFS='|' read -r n L ENVS <<< "$E"
  env $ENVS MKFHE_LIB=$PWD/$L timeout -k 10 300 python bench.py --stage evalacc --steps 1 --warmup 1 --cpu-threads 16 --paramset STD128_MKNTRU_3 --batch 8192 \
     > $O/${TAG}_c4_$n.json 2> $O/${TAG}_c4_$n.err || { echo "$n: bench failed"; tail -3 $O/${TAG}_c4_$n.err; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_c4_$n.json')); print('$n', round(d['value'],1), 'EvalAcc/s', round(d['roofline']['per_launch_us'],2), 'us/launch', 'parity', d.get('parity_checked'), d.get('parity_mismatches'))" || true
done
TAG=$TAG bash tools/gpu_r4_c5c.sh
