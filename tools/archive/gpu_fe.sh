#!/bin/bash
# serial roles on all 64 lanes (SDRG_SERIAL_FULL_EXEC variants) under co-residency, alternating with the default
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default fe7 fe2 default fe7 fe2; do
  if [ $v = default ]; then L=""; else L=$PWD/sdr-for-android-lib_amd/lib/libsdrg_$v.so; fi
  SDRG_LIB_PATH=$L timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/fe_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/fe_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/fe_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
done
