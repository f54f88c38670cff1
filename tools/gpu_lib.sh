#!/bin/bash
# tools/gpu_lib.sh -- the steps of a GPU run, one function each.  Source it and
# chain steps with && inside one gpurun command, e.g.
#
#   gpurun --timeout 1100 -- '. tools/gpu_lib.sh v3 && gtests && smoke && bench hl && \
#       bench c4gate --paramset STD128_MKNTRU_3 --stage gate --batch 8192 --steps 1'
#
# Every step runs under its own time limit, writes under gpurun_out/r5/<tag>_*, prints
# a short summary and returns non-zero on failure, so a chain stops at the first
# failing GPU step (no retries).  Steps:
#   gtests [pytest args]           the GPU suite (pytest -m gpu)
#   smoke                          __graft_entry__.smoke()
#   bench NAME [bench.py args]     one bench.py run -> NAME.json
#   ab NAME REPS "lab|lib|ENV" ... A/B of engine builds (MKFHE_LIB) / env switches, REPS
#                                  alternating rounds of one bench.py run each
#   kstats NAME [bench.py args]    rocprofv3 --kernel-trace --stats of a bench run
#   pmc NAME [bench.py args]       FETCH_SIZE and WRITE_SIZE in separate --pmc passes
#   pmcset NAME SET [bench args]   one --pmc pass of a named SQ/TCC counter set
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out/${GRUN:-r6}
mkdir -p "$O"

gtests() {
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider "$@" > "$O/${T}_pytest_gpu.txt" 2>&1
    local rc=$?
    grep -E "passed|failed|error" "$O/${T}_pytest_gpu.txt" | tail -3
    [ $rc -ne 0 ] && grep -E "FAILED|Error|error" "$O/${T}_pytest_gpu.txt" | head -20
    return $rc
}

smoke() {
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/${T}_smoke.txt" 2>&1
    local rc=$?
    tail -3 "$O/${T}_smoke.txt"
    return $rc
}

_summary() {   # one line of a bench JSON
    python3 - "$1" <<'EOF'
import json, sys
d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
r, v = d["roofline"], d.get("roofline_valu", {})
print(sys.argv[1].split("/")[-1], f"{d['value']:.1f} {d['unit']}", f"{d['ms_per_step']:.2f} ms/step",
      f"{r['per_launch_us']:.2f} us/launch", f"valu {v.get('frac', 0):.3f}", f"hbm {r['frac']:.3f}",
      "traffic", r.get("traffic"), "parity", d.get("parity_checked"), d.get("parity_mismatches"),
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
EOF
}

bench() {
    local name=$1
    shift
    timeout -k 10 700 python bench.py "$@" > "$O/${T}_$name.json" 2> "$O/${T}_$name.err"
    local rc=$?
    if [ $rc -ne 0 ]; then tail -8 "$O/${T}_$name.err"; return $rc; fi
    _summary "$O/${T}_$name.json"
}

ab() {   # ab NAME REPS "label|lib.so or -|ENV=.. ENV2=.." ... -- bench.py args after --
    local name=$1 reps=$2
    shift 2
    local entries=()
    while [ $# -gt 0 ] && [ "$1" != "--" ]; do entries+=("$1"); shift; done
    [ "$1" = "--" ] && shift
    mkdir -p "$O/${T}_ab_$name"
    local rep e lab lib envs out
    for rep in $(seq 1 "$reps"); do
        for e in "${entries[@]}"; do
            IFS='|' read -r lab lib envs <<< "$e"
            out="$O/${T}_ab_$name/$lab.$rep.json"
            if [ "$lib" = "-" ]; then lib=mkfhe_amd/lib/libmkfhe_amd.so; fi
            env $envs MKFHE_LIB="$PWD/$lib" timeout -k 10 700 python bench.py "$@" > "$out" 2> "${out%.json}.err" \
                || { echo "$lab: bench failed"; tail -5 "${out%.json}.err"; return 1; }
            _summary "$out"
        done
    done
}

kstats() {
    local name=$1
    shift
    timeout -k 10 700 rocprofv3 --kernel-trace --stats -d "$O/${T}_${name}_prof" -o run --output-format csv \
        -- python3 bench.py "$@" > "$O/${T}_${name}_prof.log" 2>&1 || { tail -20 "$O/${T}_${name}_prof.log"; return 1; }
    local f
    f=$(find "$O/${T}_${name}_prof" -name "*kernel_stats.csv" -print -quit)
    cp "$f" "$O/${T}_${name}_kernel_stats.csv"
    head -4 "$O/${T}_${name}_kernel_stats.csv" | cut -c1-200
}

# HBM traffic of the step kernel: one rocprofv3 run per counter (FETCH_SIZE alone takes
# 3 of the 4 TCC counters), the batch run as ONE stream so a dispatch is one step of
# the whole batch (the bench's bytes_per_launch), a short LWE dimension (every step
# launch has the same shape); tools/pmc_summary.py turns the CSVs into the record.
pmc() {
    local name=$1
    shift
    local cs
    for cs in FETCH_SIZE WRITE_SIZE; do
        mkdir -p "$O/${T}_pmc_$name"
        MKACC_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc $cs -d "$O/${T}_pmc_$name/$cs" -o run --output-format csv \
            -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --check-gates 4 --n-override 32 "$@" \
            > "$O/${T}_pmc_$name/$cs.log" 2>&1 || { echo "pmc $cs failed"; tail -5 "$O/${T}_pmc_$name/$cs.log"; return 1; }
    done
    echo "pmc $name done"
}

# counter sets (at most 8 SQ, 4 TCC, 2 GRBM per pass)
PMC_SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
PMC_SQ2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
PMC_L2="SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum GRBM_COUNT"
# instruction cache (SQ block on gfx950: counts toward the 8 SQ counters)
PMC_IC="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES"
pmcset() {
    local name=$1 set=$2
    shift 2
    local cs
    case $set in sq1) cs=$PMC_SQ1 ;; sq2) cs=$PMC_SQ2 ;; l2) cs=$PMC_L2 ;; ic) cs=$PMC_IC ;; *) echo "unknown set $set"; return 1 ;; esac
    mkdir -p "$O/${T}_pmc_$name"
    MKACC_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc $cs -d "$O/${T}_pmc_$name/$set" -o run --output-format csv \
        -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --check-gates 4 --n-override 32 "$@" \
        > "$O/${T}_pmc_$name/$set.log" 2>&1 || { echo "pmc $set failed"; tail -5 "$O/${T}_pmc_$name/$set.log"; return 1; }
    echo "pmcset $name $set done"
}
