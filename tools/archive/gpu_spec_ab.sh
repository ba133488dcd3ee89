#!/bin/bash
# A/B of the spectrum16k kernel in one session: the product library vs lib/libsdrg_${B:-specold}.so, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
for i in 1 2 3; do
  for lib in libsdrg.so libsdrg_${B:-specold}.so; do
    SDRG_LIB_PATH=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-labelled ${ARGS:-} > gpurun_out/ab.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['kernel_ms']['spectrum_ms'], d['kernel_ms']['ssb_ms'], d.get('roofline_isolated',{}).get('achieved'))"
  done
done
