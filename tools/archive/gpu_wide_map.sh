#!/bin/bash
# Wide statistics (BASELINE configs[4], 65536 / 200 kHz): placement-aware chain role (SDRG_WIDE_MAP) and chain issue
# priority (SDRG_WIDE_PRIO), lab builds against the product; wave placement probe first.
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
timeout -k 10 60 tools/lab/hwid_probe > gpurun_out/wmap_probe.log 2>&1 || { echo "probe failed"; cat gpurun_out/wmap_probe.log; exit 1; }
cat gpurun_out/wmap_probe.log
for v in map1p2; do SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_stats_exact.py tests/test_gpu_stats_geometry.py -m gpu -x -q --timeout 120 --timeout-method thread -k "200 or 65536" > gpurun_out/wmap_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 gpurun_out/wmap_tests_$v.log; exit 1; }; tail -n 1 gpurun_out/wmap_tests_$v.log; done
for v in stamps stampsmap; do SDRG_LIB_PATH=$L/libsdrg_$v.so timeout -k 10 120 python tools/kernel_lab.py --stages spectrum+stats --n 65536 --fmt CS16 --streams 1024 --focus 200 --calls 3 > gpurun_out/wmap_st_$v.log 2>&1 || { echo "stamps $v failed"; tail gpurun_out/wmap_st_$v.log; exit 1; }; echo "== $v"; cat gpurun_out/wmap_st_$v.log; done
run() {
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled --config c5 --focus 200 > gpurun_out/wmap_$1_$2.json 2> gpurun_out/wmap_$1_$2.err || { echo "bench $1 failed"; tail -5 gpurun_out/wmap_$1_$2.err; exit 1; }
  echo "$1 $2 $(tail -n 1 gpurun_out/wmap_$1_$2.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run product $r && run map1 $r && run map1p2 $r && run p2 $r || exit 1; done
