#!/bin/bash
# statistics parity, then c2 / c5 lines: product library vs lib/libsdrg_${B:-statsold}.so, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_any_n.py tests/test_gpu_edges.py tests/test_gpu_engine_api.py tests/test_gpu_multi_rank.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/stats_parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/stats_parity.log; exit 1; }
tail -1 gpurun_out/stats_parity.log
L=$PWD/sdr-for-android-lib_amd/lib
for i in 1 2; do
  for lib in libsdrg.so libsdrg_${B:-statsold}.so; do
    for a in "--config c2" "--config c5 --focus 5" ""; do
      SDRG_LIB_PATH=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-labelled $a > gpurun_out/sab.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/sab.log; exit 1; }
      tail -1 gpurun_out/sab.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print('$lib', '${a:-c3}', d['value'], d['ms_per_step'], k['spectrum_ms'], k['stats_ms'], k['ssb_ms'])"
    done
  done
done
