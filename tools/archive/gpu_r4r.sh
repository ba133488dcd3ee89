#!/bin/bash
# round 4: the SSB stream's end marker completed by the pipeline kernel's own dispatch (hipExtLaunchKernel stop event,
# extstop) instead of a marker packet after it (extbase): GPU tests on extstop, then the c3 lines alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$D/libsdrg_extstop.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_engine_api.py tests/test_gpu_pulse.py tests/test_gpu_ssb_processor.py > gpurun_out/r4r_tests.log 2>&1 || { tail -30 gpurun_out/r4r_tests.log; exit 1; }
echo "extstop tests: $(tail -1 gpurun_out/r4r_tests.log)"
for i in 1 2; do
  for v in extbase extstop; do
    SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-labelled > gpurun_out/r4r.json 2>/dev/null || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r4r.json')); s=d['ssb_latency_floor']; print(d['value'], d['ms_per_step'], d['kernel_ms'], s['ssb_ms_alone'], s['ssb_ms_coresident'])")"
    SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-labelled > gpurun_out/r4r20.json 2>/dev/null || exit 1
    echo "$v 20-step $(python3 -c "import json; d=json.load(open('gpurun_out/r4r20.json')); print(d['value'], d['ms_per_step'])")"
  done
done
