#!/bin/bash
# default bench line with each named variant library ("" = the product), alternating, twice
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for n in "$@"; do
    lib=""; [ "$n" = product ] || lib=sdr-for-android-lib_amd/lib/libsdrg_$n.so
    SDRG_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-labelled > gpurun_out/libs_ab.log 2>&1 || exit 1
    echo "$n $(tail -1 gpurun_out/libs_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
