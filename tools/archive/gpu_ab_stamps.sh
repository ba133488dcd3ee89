#!/bin/bash
# A/B of two lab variants (tools/build_variant.sh NAME): the GPU suite on A, per-role SSB stamps of both, then the
# default bench line alternately A, B, A, B (one box)
export TMPDIR=/tmp
A=$1; B=$2
LA=sdr-for-android-lib_amd/lib/libsdrg_$A.so; LB=sdr-for-android-lib_amd/lib/libsdrg_$B.so
mkdir -p gpurun_out
SDRG_LIB_PATH=$LA timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$A.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_$A.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests_$A.log | head -20; exit 1; }
for v in $A $B; do
  SDRG_LIB_PATH=sdr-for-android-lib_amd/lib/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/stamps_$v.log 2>&1 || exit 1
  echo "== stamps $v"; grep stamps gpurun_out/stamps_$v.log | tail -12 | cut -c1-100
done
for i in 1 2; do
  for v in $A $B; do
    SDRG_LIB_PATH=sdr-for-android-lib_amd/lib/libsdrg_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-labelled > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['ssb_latency_floor']['ssb_ms_alone'])")"
  done
done
