#!/bin/bash
# round 4: the wide statistics kernels (multi-frame vs single-frame, LDS-only chunk barrier vs __syncthreads) on
# BASELINE configs[4] at 200 kHz, alternating on one box, after the statistics GPU tests on the product library
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stats_geometry.py \
    tests/test_gpu_stats_exact.py tests/test_gpu_engine_api.py > gpurun_out/r4c_tests.log 2>&1 \
    || { grep -E "FAIL|Error|assert" gpurun_out/r4c_tests.log | head -30; tail -5 gpurun_out/r4c_tests.log; exit 1; }
tail -1 gpurun_out/r4c_tests.log
for i in 1 2; do
  for v in prodlab:0 prodlab:1 nobar:0 nobar:1; do
    lib=${v%%:*}; single=${v##*:}
    if [ $single = 1 ]; then export SDRG_WIDE_SINGLE=1; else unset SDRG_WIDE_SINGLE; fi
    SDRG_LIB_PATH=sdr-for-android-lib_amd/lib/libsdrg_$lib.so timeout -k 10 200 python bench.py --config c5 --focus 200 --steps 100 --warmup 20 > gpurun_out/r4c_$lib$single.json 2>/dev/null || exit 1
    echo "$lib single=$single $(python3 -c "import json; d=json.load(open('gpurun_out/r4c_$lib$single.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
