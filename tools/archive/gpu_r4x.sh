#!/bin/bash
# round 4: SSB role-to-wave maps (SDRG_PIPE_MAP, wave w runs on SIMD w % 4) under the per-role priorities; c3 line,
# lab build, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in $(seq 1 ${ROUNDS:-2}); do
  for m in ${MAPS:-7B984A653210}; do
    SDRG_PIPE_MAP=$m SDRG_LIB_PATH=$D/libsdrg_lab.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-labelled --no-cpu-baseline > gpurun_out/r4x.json 2>/dev/null || exit 1
    echo "map $m $(python3 -c "import json; d=json.load(open('gpurun_out/r4x.json')); print(d['value'], d['ms_per_step'], d['kernel_ms']['ssb_ms'])")"
  done
done
