#!/bin/bash
# SSB pipeline capped at 80 VGPRs / 84.5 KiB LDS (variants co16, co) so a spectrum workgroup co-resides with it:
# parity of the variant, then bench lines for default / co16 / co
export TMPDIR=/tmp
mkdir -p gpurun_out
SDRG_LIB_PATH=$PWD/sdr-for-android-lib_amd/lib/libsdrg_co16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cores_parity.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/cores_parity.log; exit 1; }
tail -1 gpurun_out/cores_parity.log
for v in default co16 co default co16; do
  if [ $v = default ]; then L=""; else L=$PWD/sdr-for-android-lib_amd/lib/libsdrg_$v.so; fi
  SDRG_LIB_PATH=$L timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/cores_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/cores_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/cores_$v.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["roofline"]["frac"], d["roofline_isolated"]["frac"])')"
done
