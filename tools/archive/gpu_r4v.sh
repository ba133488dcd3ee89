#!/bin/bash
# round 4: SSB helper waves' issue priority (SDRG_PIPE_PRIO mask of high-priority waves: 0x7 = the serial roles, the
# product; 0xFFF = every SSB wave) beside the spectrum and the asynchronous statistics, lab build, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in $(seq 1 ${ROUNDS:-2}); do
  for m in ${MASKS:-0x7 0xFFF 0xF07}; do
    SDRG_PIPE_PRIO=$m SDRG_LIB_PATH=$D/libsdrg_lab.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-labelled --no-cpu-baseline > gpurun_out/r4v.json 2>/dev/null || exit 1
    echo "prio $m $(python3 -c "import json; d=json.load(open('gpurun_out/r4v.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
