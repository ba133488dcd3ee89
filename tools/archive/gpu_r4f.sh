#!/bin/bash
# round 4: multi-frame wide statistics variants (prodlab: before the kmax change; km: kmax; map1: kmax + chain SIMD
# isolated) vs the single-frame kernel: parity of the product library, stamps, alone, and the configs[4] 200 kHz line
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stats_geometry.py tests/test_gpu_stats_exact.py > gpurun_out/r4f_tests.log 2>&1 || { tail -20 gpurun_out/r4f_tests.log; exit 1; }
tail -1 gpurun_out/r4f_tests.log
SDRG_LIB_PATH=$D/libsdrg_map1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stats_geometry.py -k partial > gpurun_out/r4f_tests_map1.log 2>&1 || { tail -20 gpurun_out/r4f_tests_map1.log; exit 1; }
tail -1 gpurun_out/r4f_tests_map1.log
bash tools/gpu_r4e.sh mwst0 mwst || exit 1
for i in 1 2; do
  SDRG_LIB_PATH=$D/libsdrg_prodlab.so SDRG_WIDE_SINGLE=1 timeout -k 10 60 python tools/lab/stats_time.py || exit 1
  for v in prodlab km map1; do SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 60 python tools/lab/stats_time.py || exit 1; done
done
for i in 1 2; do
  for v in prodlab:1 km:0 map1:0; do
    lib=${v%%:*}; single=${v##*:}
    if [ $single = 1 ]; then export SDRG_WIDE_SINGLE=1; else unset SDRG_WIDE_SINGLE; fi
    SDRG_LIB_PATH=$D/libsdrg_$lib.so timeout -k 10 200 python bench.py --config c5 --focus 200 --steps 100 --warmup 20 > gpurun_out/r4f.json 2>/dev/null || exit 1
    echo "$lib single=$single $(python3 -c "import json; d=json.load(open('gpurun_out/r4f.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
