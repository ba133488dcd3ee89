#!/bin/bash
# r6f: the low-pass adds with the running sum as src1 (lab "src1"; "copsrc1" = the same on four full-EXEC copies):
# SSB parity, the SSB stage's low-pass loop (stamps), then the c3 line alternating against the product.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
for v in src1 copsrc1; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py \
    > gpurun_out/r6f_tests_$v.log 2>&1 || { echo "$v tests FAILED"; tail -40 gpurun_out/r6f_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r6f_tests_$v.log)"
done
for v in lab src1 copsrc1 lab src1 copsrc1; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 timeout -k 10 200 python tools/lab/step_once.py ${v}_ssb 4 > gpurun_out/r6f_stamps_${v}_ssb.log 2>&1 || { echo "stamps $v failed"; tail gpurun_out/r6f_stamps_${v}_ssb.log; exit 1; }
  echo "$v: $(grep 'wave 1 LPF' gpurun_out/r6f_stamps_${v}_ssb.log | tail -1 | sed 's/.*steady/steady/') | $(grep ms/step gpurun_out/r6f_stamps_${v}_ssb.log)"
done
tools/ab.sh -r 2 -o r6f base src1 -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled
