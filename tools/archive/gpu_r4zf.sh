#!/bin/bash
# round 4: SDRG_MW_WREF=3 or 1 (wref3 / wref1: reference-window producer lanes per focus lane) against 2 (base), after the
# folded log table made the reference logs cheaper: the wide statistics GPU tests on $W, then stats alone and c5 200 kHz
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
W=${1:-wref3}
SDRG_LIB_PATH=$D/libsdrg_$W.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_libm_exact.py > gpurun_out/r4zf_tests.log 2>&1 || { tail -30 gpurun_out/r4zf_tests.log; exit 1; }
tail -2 gpurun_out/r4zf_tests.log
for i in 1 2 3; do
  for v in base $W; do
    echo "$v stats alone: $(SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 120 python tools/lab/stats_time.py 65536 200 1024 30 2>/dev/null | tail -1)"
    SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --config c5 --focus 200 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r4zf.json 2>/dev/null || exit 1
    echo "$v 200 kHz $(python3 -c "import json; d=json.load(open('gpurun_out/r4zf.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
