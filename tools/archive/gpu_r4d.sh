#!/bin/bash
# round 4: the multi-frame wide statistics kernel: parity (product library), then alone (tools/lab/stats_time.py) and in
# the configs[4] 200 kHz line, against the single-frame kernel (lab build, SDRG_WIDE_SINGLE=1), alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stats_geometry.py \
    tests/test_gpu_stats_exact.py tests/test_gpu_parity.py tests/test_gpu_engine_api.py tests/test_gpu_any_n.py > gpurun_out/r4d_tests.log 2>&1 \
    || { grep -E "FAIL|Error|assert" gpurun_out/r4d_tests.log | head -30; tail -5 gpurun_out/r4d_tests.log; exit 1; }
tail -1 gpurun_out/r4d_tests.log
L=sdr-for-android-lib_amd/lib/libsdrg_prodlab.so
for i in 1 2; do
  SDRG_LIB_PATH=$L SDRG_WIDE_SINGLE=1 timeout -k 10 60 python tools/lab/stats_time.py || exit 1
  SDRG_LIB_PATH=$L timeout -k 10 60 python tools/lab/stats_time.py || exit 1
done
for i in 1 2; do
  for single in 1 0; do
    if [ $single = 1 ]; then export SDRG_WIDE_SINGLE=1; else unset SDRG_WIDE_SINGLE; fi
    SDRG_LIB_PATH=$L timeout -k 10 200 python bench.py --config c5 --focus 200 --steps 100 --warmup 20 > gpurun_out/r4d_c5_$single.json 2>/dev/null || exit 1
    echo "single=$single $(python3 -c "import json; d=json.load(open('gpurun_out/r4d_c5_$single.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
