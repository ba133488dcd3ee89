#!/bin/bash
# (nfold: a temporary copy of stats.hip; not kept)
# round 4: the narrow statistics' per-bin logs through the folded table too (nfold: built from a copy of stats.hip whose
# narrow kernel loads s_logf_fold and calls db_fold for its bins) against fold (wide kernels only): narrow statistics
# GPU tests on nfold, then the c3 default line, c2 and configs[4] 5 kHz, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$D/libsdrg_nfold.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_parity.py > gpurun_out/r4zd_tests.log 2>&1 || { tail -30 gpurun_out/r4zd_tests.log; exit 1; }
tail -1 gpurun_out/r4zd_tests.log
for i in 1 2; do
  for v in fold nfold; do
    for c in "" "--config c2" "--config c5 --focus 5"; do
      SDRG_LIB_PATH=$D/libsdrg_$v.so timeout -k 10 200 python bench.py $c --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r4zd.json 2>/dev/null || exit 1
      echo "$v [$c] $(python3 -c "import json; d=json.load(open('gpurun_out/r4zd.json')); print(d['value'], d['ms_per_step'])")"
    done
  done
done
