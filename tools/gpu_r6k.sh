#!/bin/bash
# r6k: does the serial waves' partial EXEC cap the low-pass loop?  "ser3" = the DC and AGC chunks with their VALU on all
# 64 lanes (SDRG_SERIAL_SPLIT=5); "sgs3" = that plus the low-pass loop with full-EXEC VALU and global-store outputs.
# SSB parity on both, in-situ stamps, c3 line alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
for v in ser3 sgs3; do
  SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_pulse.py tests/test_gpu_ssb_schedule.py tests/test_gpu_ssb_variant.py tests/test_gpu_edges.py \
    > gpurun_out/r6k_tests_$v.log 2>&1 || { echo "$v tests FAILED"; tail -40 gpurun_out/r6k_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r6k_tests_$v.log)"
done
for spec in lab:0 ser3:0 sgs3:0 sgs3:0xFFD ser3:0 sgs3:0 lab:0; do
  v=${spec%%:*}; m=${spec#*:}
  SDRG_LIB_PATH=$L/libsdrg_$v.so SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$m timeout -k 10 200 python tools/lab/step_once.py ${v}_$m 4 > gpurun_out/r6k_stamps_${v}_$m.log 2>&1 || { echo "stamps $spec failed"; tail gpurun_out/r6k_stamps_${v}_$m.log; exit 1; }
  echo "$spec: $(grep 'wave 1 LPF' gpurun_out/r6k_stamps_${v}_$m.log | tail -1 | sed 's/.*steady/steady/') | $(grep ms/step gpurun_out/r6k_stamps_${v}_$m.log)"
done
grep -v "abs entry" gpurun_out/r6k_stamps_sgs3_0.log | grep "wave" | tail -12
tools/ab.sh -r 2 -o r6k base ser3 sgs3 -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled
