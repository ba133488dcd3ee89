#!/bin/bash
# r6a: the barrier-free SSB pipeline (SDRG_PIPE_FLAGS=1, lab build "flags") — SSB parity first, then alternating
# A/B against the product, then per-role stamps of both (lab builds "lab" and "flags").
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$L/libsdrg_flags.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py tests/test_gpu_ssb_variant.py \
  > gpurun_out/r6a_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/r6a_tests.log; exit 1; }
tail -2 gpurun_out/r6a_tests.log
tools/ab.sh -r 2 -o r6a base flags -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled || exit 1
for v in lab flags; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 200 python tools/lab/step_once.py $v 31 > gpurun_out/r6a_stamps_$v.log 2>&1 || { echo "stamps $v failed"; tail gpurun_out/r6a_stamps_$v.log; exit 1; }
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 200 python tools/lab/step_once.py ${v}_ssb 4 > gpurun_out/r6a_stamps_${v}_ssb.log 2>&1 || { echo "stamps $v ssb failed"; exit 1; }
  grep -v "abs entry" gpurun_out/r6a_stamps_$v.log | tail -15
  grep -v "abs entry" gpurun_out/r6a_stamps_${v}_ssb.log | tail -15
done
