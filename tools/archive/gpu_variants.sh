#!/bin/bash
# time diagnostic library variants (lib/libsdrg_*.so) on given stages: VARIANTS="a b" STAGES="spectrum all"
export TMPDIR=/tmp
for v in default ${VARIANTS}; do
  if [ $v = default ]; then L=""; else L=sdr-for-android-lib_amd/lib/libsdrg_$v.so; fi
  for st in ${STAGES:-spectrum}; do
    SDRG_LIB_PATH=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --stages $st > gpurun_out/var_${v}_$st.log 2>&1 || { echo "variant $v $st failed"; tail -5 gpurun_out/var_${v}_$st.log; exit 1; }
    echo "$v $st: $(tail -1 gpurun_out/var_${v}_$st.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"])')"
  done
done
