#!/bin/bash
# one call: lat-kernel stress (old DG=3 build vs the current library), the full check
# of the current library (tools/gpu_check.sh), then the batch-kernel timing A/B
# usage: tools/gpu_round.sh TAG OLD.so [AB LIBS...]
TAG=$1; OLD=$2; shift 2
bash tools/gpu_lat_ab.sh $TAG 300 $OLD,mkfhe_amd/lib/libmkfhe_amd.so || exit $?
bash tools/gpu_check.sh $TAG || exit $?
if [ $# -gt 0 ]; then MKACC_LAT=0 PARITY_K=logB7 bash tools/gpu_ab.sh $TAG "$@" || exit $?; fi
exit 0
