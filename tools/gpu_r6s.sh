#!/bin/bash
# r6s: the lab-code pruning (ssb.hip, stats.hip, spectrum.hip, the generated header) against the previous product
# library (libsdrg_prev.so, built from the commit before): full GPU suite on the new product, the wide statistics alone
# (the multi-frame kernel's code changed shape), then the bench A/B with the labelled lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6s_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/r6s_smoke.log; exit 1; }
tail -1 gpurun_out/r6s_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6s_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -30 gpurun_out/r6s_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r6s_gpu_tests.log
for r in 1 2; do
  for v in prev base; do
    lib=$L/libsdrg.so; [ $v != base ] && lib=$L/libsdrg_$v.so
    SDRG_LIB_PATH=$lib timeout -k 10 120 python tools/lab/stats_time.py 65536 200 1024 30 > gpurun_out/r6s_st_${v}_$r.log 2>&1 || { echo "stats_time $v failed"; tail gpurun_out/r6s_st_${v}_$r.log; exit 1; }
    echo "wide stats $v: $(tail -1 gpurun_out/r6s_st_${v}_$r.log)"
  done
done
bash tools/ab.sh -r 2 -o r6s prev base -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline
