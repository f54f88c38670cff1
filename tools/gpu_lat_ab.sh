#!/bin/bash
# lat-kernel stress (A/B of the VCC fix), then batch-kernel timing A/B with the small-batch kernel off
# usage: tools/gpu_lat_ab.sh TAG ITERS STRESS_LIBS(comma-separated) [AB LIBS...]
TAG=$1; ITERS=$2; SL=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in ${SL//,/ }; do
  MKFHE_LIB=$PWD/$L timeout -k 10 300 python -u tools/lat_stress.py $ITERS > gpurun_out/lat_${TAG}_$(basename $L .so).txt 2>&1
  rc=$?; tail -1 gpurun_out/lat_${TAG}_$(basename $L .so).txt
  [ $rc -ne 0 ] && { echo "lat stress rc=$rc"; exit $rc; }
done
if [ $# -gt 0 ]; then MKACC_LAT=0 PARITY_K="${PARITY_K:-logB7}" bash tools/gpu_ab.sh $TAG "$@" || exit $?; fi
exit 0
