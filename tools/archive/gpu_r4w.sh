#!/bin/bash
# round 4: the spectrum waves at issue priority 1 (sp1) beside the SSB pipeline whose recurrences (3), DES0-DES2 and
# loader (2) sit above it, against priority 0 (sp0); c3 line, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in 1 2 3; do
  for v in sp0 sp1; do
    SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-labelled --no-cpu-baseline > gpurun_out/r4w.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r4w.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
