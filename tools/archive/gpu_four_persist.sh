#!/bin/bash
# Four-step FFT (32768 / 65536): persistent kernels with next-tile prefetch (SDRG_FOUR_PERSIST, lab build "fp")
# against the product: parity tests on the lab build, then alternating configs[4] bench lines (5 and 200 kHz focus)
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/sdr-for-android-lib_amd/lib
SDRG_LIB_PATH=$L/libsdrg_fp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stats_exact.py tests/test_gpu_any_n.py -m gpu -x -q --timeout 120 --timeout-method thread -k "65536 or 32768 or golden or async or pipelined" > gpurun_out/fp_tests.log 2>&1 || { echo "tests fp failed"; tail -30 gpurun_out/fp_tests.log; exit 1; }
tail -n 1 gpurun_out/fp_tests.log
run() {
  lib=""; [ "$1" != product ] && lib=$L/libsdrg_$1.so
  SDRG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-labelled --config c5 --focus $3 > gpurun_out/fp_$1_$2_$3.json 2> gpurun_out/fp_$1_$2_$3.err || { echo "bench $1 failed"; tail -5 gpurun_out/fp_$1_$2_$3.err; exit 1; }
  echo "$1 $2 focus $3: $(tail -n 1 gpurun_out/fp_$1_$2_$3.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"])')"
}
for r in a b; do run product $r 5 && run fp $r 5 && run product $r 200 && run fp $r 200 || exit 1; done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fp_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kernel_lab.py --stages spectrum --n 65536 --fmt CS16 --streams 1024 --calls 10 > $GRAFT_REPO_ROOT/gpurun_out/fp_prof.log 2>&1 || { echo "prof product failed"; exit 1; }
SDRG_LIB_PATH=$L/libsdrg_fp.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fp_prof_fp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kernel_lab.py --stages spectrum --n 65536 --fmt CS16 --streams 1024 --calls 10 > $GRAFT_REPO_ROOT/gpurun_out/fp_prof_fp.log 2>&1 || { echo "prof fp failed"; exit 1; }
cd $GRAFT_REPO_ROOT; for d in fp_prof fp_prof_fp; do echo "== $d"; f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); grep -i "four_step" $f | cut -d, -f1-6; done
