#!/bin/bash
# sample GPU power and shader clock (read-only rocm-smi) while the bench runs, per mode
export TMPDIR=/tmp
mkdir -p gpurun_out/power
for F in 0 1; do
  ( for i in $(seq 1 40); do rocm-smi --showpower --showclocks --json 2>/dev/null; sleep 0.25; done ) \
      > gpurun_out/power/smi_$F.jsonl &
  SMI=$!
  MKACC_FUSED=$F timeout -k 10 300 python bench.py --steps 6 --warmup 1 --cpu-baseline 0 "$@" \
      > gpurun_out/power/bench_$F.json 2> gpurun_out/power/bench_$F.err
  rc=$?
  kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
  [ $rc -ne 0 ] && { tail -3 gpurun_out/power/bench_$F.err; exit $rc; }
  python3 - "$F" <<'EOF'
import json, re, sys
F = sys.argv[1]
d = json.load(open(f"gpurun_out/power/bench_{F}.json"))
txt = open(f"gpurun_out/power/smi_{F}.jsonl").read()
pw = [float(x) for x in re.findall(r'"(?:Current Socket Graphics Package Power|Average Graphics Package Power) \(W\)": "([0-9.]+)"', txt)]
sc = [int(x) for x in re.findall(r'"sclk clock speed:": "\((\d+)Mhz\)"', txt)]
top = lambda v: sorted(v)[len(v) // 2:] if v else []
print(f"fused={F} value={d['value']:.1f} power_W(max,median-top-half)={max(pw) if pw else None},"
      f"{top(pw)[len(top(pw))//2] if pw else None} sclk_MHz(min,max)={min(sc) if sc else None},{max(sc) if sc else None}")
EOF
done
