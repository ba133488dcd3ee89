#!/bin/bash
# r6q: persistent spectrum workgroups taking frames from a device counter (lab build dyn, SDRG_K16_DYN=1) against the
# product's grid stride: spectrum hashes (same bits), parity tests, spectrum alone, then the bench A/B with the labelled
# configs[1] lines (both statistics schedules).  (First run faulted: the slot was a static __shared__ int, which moved
# the dynamic LDS off offset 0 and exch1's base-folded XOR addresses onto it; now a slot after the tables.)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
for v in dyn base; do
  lib=$L/libsdrg.so; [ $v != base ] && lib=$L/libsdrg_$v.so
  for f in cs8 cs16 cu8 cf32; do
    SDRG_LIB_PATH=$lib timeout -k 10 120 python tools/lab/spec_time.py 16384 $f 4096 100 > gpurun_out/r6q_spec_${v}_$f.log 2>&1 || { echo "spec_time $v $f failed"; tail gpurun_out/r6q_spec_${v}_$f.log; exit 1; }
    echo "$v $f: $(tail -1 gpurun_out/r6q_spec_${v}_$f.log)"
  done
done
bash tools/ab.sh -r 2 -o r6q -t "tests/test_gpu_parity.py tests/test_gpu_edges.py" base dyn -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline
