#!/bin/bash
# r6d: (1) what slows the low-pass wave in situ: the SSB stage alone (lab build "lab", stamps) with one helper role's
# work skipped at a time (SDRG_PIPE_SKIP, wrong results, timing only); (2) VERDICT r5 item 2's fusion cost, lower bound:
# the spectrum kernel with 384 extra packed FMAs per thread and frame (lab "fuse384", the VALU a fused narrow-statistics
# tail adds) against the product, alone and in the configs[1] line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
for m in 0 0x90 0xF00 0x20 0x40 0x8 0x4 0x1 0xFFD 0; do
  SDRG_LIB_PATH=$L/libsdrg_lab.so SDRG_PIPE_STAMPS=1 SDRG_PIPE_SKIP=$m timeout -k 10 200 python tools/lab/step_once.py skip_$m 4 \
    > gpurun_out/r6d_skip_$m.log 2>&1 || { echo "skip $m failed"; tail gpurun_out/r6d_skip_$m.log; exit 1; }
  echo "skip $m: $(grep 'wave 1 LPF' gpurun_out/r6d_skip_$m.log | tail -1 | sed 's/.*steady/steady/') | $(grep ms/step gpurun_out/r6d_skip_$m.log)"
done
for r in 1 2; do
  for v in fuse384 product; do
    if [ $v = product ]; then lib=$L/libsdrg.so; else lib=$L/libsdrg_$v.so; fi
    SDRG_LIB_PATH=$lib timeout -k 10 120 python tools/lab/spec_time.py 16384 cs8 4096 200 || exit 1
  done
done
tools/ab.sh -r 2 -o r6d base fuse384 -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline
