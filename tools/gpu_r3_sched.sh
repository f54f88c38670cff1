#!/bin/bash
# round 3: step2 dg = 3 unit built with other machine-scheduler strategies (spill-free at 256 VGPRs)
# against the same unit built with the default strategy (6 spilled VGPRs); headline EvalAcc, ABAB
export TMPDIR=/tmp
bash tools/gpu_ab_matrix.sh sched "ctl|mkfhe_amd/lib/variants/ctl.so|" "mmc|mkfhe_amd/lib/variants/mmc.so|" "ilp|mkfhe_amd/lib/variants/ilp.so|"
