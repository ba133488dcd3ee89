#!/bin/bash
# Statistics variants, alternating: the product (dB via the glibc log10f restatement, focus dB only near the
# largest power), lab "glibc" (the restatement on every focus bin), lab "ocml" (round 2: ocml's log10f).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py tests/test_gpu_parity.py tests/test_gpu_any_n.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sab_tests.log; exit 1; }
tail -1 gpurun_out/sab_tests.log
L=$PWD/sdr-for-android-lib_amd/lib
run() {  # variant tag [extra]
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-labelled $3 > gpurun_out/sab_$1_$2.json 2> gpurun_out/sab_$1_$2.err || { echo "bench $1 failed"; tail -5 gpurun_out/sab_$1_$2.err; exit 1; }
  echo "$1 $2 $(tail -1 gpurun_out/sab_$1_$2.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run product $r && run glibc $r && run ocml $r || exit 1; done
for r in c5a c5b; do run product $r "--config c5 --focus 200" && run glibc $r "--config c5 --focus 200" && run ocml $r "--config c5 --focus 200" || exit 1; done
