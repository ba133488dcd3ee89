#!/bin/bash
# round 4: everything but the statistics one issue-priority level up (spectrum 1, SSB helpers 1, DES0-DES2 and loader 2,
# recurrences 3; statistics 0: sp1lab + mask 0x806A55BF) against the product's levels (lab + 0x802A00BF); c3, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in 1 2 3; do
  for v in lab:0x802A00BF sp1lab:0x806A55BF; do
    lib=${v%%:*}; m=${v##*:}
    SDRG_PIPE_PRIO=$m SDRG_LIB_PATH=$D/libsdrg_$lib.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-labelled --no-cpu-baseline > gpurun_out/r4z.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r4z.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
