#!/bin/bash
export TMPDIR=/tmp
TAG=$TAG bash tools/gpu_r4_base.sh && TAG=$TAG bash tools/gpu_r4_cfg4.sh
