#!/bin/bash
# r6e: the low-pass loop on all 64 lanes as four copies of the 16 streams (lab "copies", SDRG_LPF_COPIES=1): SSB parity,
# the SSB stage's stamps, then the c3 line alternating against the product.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$L/libsdrg_copies.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py tests/test_gpu_ssb_variant.py \
  > gpurun_out/r6e_tests_copies.log 2>&1 || { echo "copies tests FAILED"; tail -40 gpurun_out/r6e_tests_copies.log; exit 1; }
echo "copies: $(tail -1 gpurun_out/r6e_tests_copies.log)"
for v in lab copies lab copies; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 200 python tools/lab/step_once.py ${v}_ssb 4 > gpurun_out/r6e_stamps_${v}_ssb.log 2>&1 || { echo "stamps $v failed"; tail gpurun_out/r6e_stamps_${v}_ssb.log; exit 1; }
  echo "$v: $(grep 'wave 1 LPF' gpurun_out/r6e_stamps_${v}_ssb.log | tail -1 | sed 's/.*steady/steady/') | $(grep ms/step gpurun_out/r6e_stamps_${v}_ssb.log)"
done
grep -v "abs entry" gpurun_out/r6e_stamps_copies_ssb.log | tail -13
tools/ab.sh -r 2 -o r6e base copies -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled
