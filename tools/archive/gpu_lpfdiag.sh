#!/bin/bash
# SSB per-role cycles (stamps) with the product library and with the LPF recurrence on register data (no LDS)
export TMPDIR=/tmp
run() { SDRG_LIB_PATH=$3 SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag.log 2>&1 || exit 1; echo "== skip $1 $2"; grep stamps gpurun_out/ssbdiag.log | tail -12; }
run 0 "product" "" || exit 1
run 0 "all, lpf no lds" sdr-for-android-lib_amd/lib/libsdrg_lpfnolds.so || exit 1
run 0xFFD "LPF only, no lds" sdr-for-android-lib_amd/lib/libsdrg_lpfnolds.so || exit 1
run 0xFFD "LPF only, product" "" || exit 1
