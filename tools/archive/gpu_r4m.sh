#!/bin/bash
# round 4: co-residency of the wide multi-frame statistics with the next call's four-step FFT (configs[4] 200 kHz):
# VGPRs capped at 96 (v96: a kernel-B workgroup fits beside it; v96lg7: 2^7-bin chunks, so a kernel-A one fits too)
# against the product build (mwbase); statistics alone and the c5/200 line, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for v in v96 v96lg7; do
  SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_stats_geometry.py tests/test_gpu_stats_exact.py > gpurun_out/r4m_tests_$v.log 2>&1 || { tail -20 gpurun_out/r4m_tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r4m_tests_$v.log)"
done
for i in 1 2; do
  for v in mwbase v96 v96lg7; do
    echo "$v alone: $(SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 60 python tools/lab/stats_time.py 65536 200 1024 30)" || exit 1
    SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --config c5 --focus 200 --steps 100 --warmup 20 > gpurun_out/r4m.json 2>/dev/null || exit 1
    echo "$v c5/200 $(python3 -c "import json; d=json.load(open('gpurun_out/r4m.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
