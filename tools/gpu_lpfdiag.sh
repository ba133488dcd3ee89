#!/bin/bash
export TMPDIR=/tmp
run() { SDRG_LIB_PATH=$3 SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag.log 2>&1 || exit 1; echo "== skip $1 $2"; grep stamps gpurun_out/ssbdiag.log | tail -12 | awk '{printf "%s %s work %s loop %s\n", $4, $5, $7, $10}' | head -3; }
run 0 "all, lpf no lds" sdr-for-android-lib_amd/lib/libsdrg_lpfnolds.so
run 0xFFD "LPF only, no lds" sdr-for-android-lib_amd/lib/libsdrg_lpfnolds.so
