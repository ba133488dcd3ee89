#!/bin/bash
# round 4: multi-frame wide statistics (parity, then configs[4] 200 kHz A/B against the single-frame kernel), and the
# spread serial-lane map A/B (tools/gpu_ab_stamps.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stats_geometry.py \
    tests/test_gpu_stats_exact.py tests/test_gpu_parity.py tests/test_gpu_engine_api.py tests/test_gpu_any_n.py > gpurun_out/r4b_tests.log 2>&1 \
    || { grep -E "FAIL|Error|assert" gpurun_out/r4b_tests.log | head -30; tail -5 gpurun_out/r4b_tests.log; exit 1; }
tail -1 gpurun_out/r4b_tests.log
L=sdr-for-android-lib_amd/lib/libsdrg_prodlab.so
for i in 1 2; do
  for single in 1 0; do
    if [ $single = 1 ]; then export SDRG_WIDE_SINGLE=1; else unset SDRG_WIDE_SINGLE; fi
    SDRG_LIB_PATH=$L timeout -k 10 200 python bench.py --config c5 --focus 200 --steps 100 --warmup 20 > gpurun_out/r4b_c5_$single.json 2>/dev/null || exit 1
    echo "single=$single $(python3 -c "import json; d=json.load(open('gpurun_out/r4b_c5_$single.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
unset SDRG_WIDE_SINGLE
bash tools/gpu_ab_stamps.sh spread prodlab
