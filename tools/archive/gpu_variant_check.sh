#!/bin/bash
# a variant library (tools/build_variant.sh NAME): the GPU suite on it, per-role SSB cycles, then the default bench
# line with it and with the product library alternately (A/B on one box)
export TMPDIR=/tmp
V=sdr-for-android-lib_amd/lib/libsdrg_$1.so
mkdir -p gpurun_out
SDRG_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$1.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_$1.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/gpu_tests_$1.log | head -20; exit 1; }
SDRG_LIB_PATH=$V SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/ssbdiag.log 2>&1 || exit 1
grep stamps gpurun_out/ssbdiag.log | tail -12 | cut -c1-90
for i in 1 2; do
  for lib in "$V" ""; do
    SDRG_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-labelled > gpurun_out/bench_ab.log 2>&1 || exit 1
    echo "lib=${lib:-product} $(tail -1 gpurun_out/bench_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'])")"
  done
done
