#!/bin/bash
# Round 3: 32-stream SSB workgroups on half the CUs (product) against the 16-stream co-resident pipeline (lab pg16)
# and the even/odd CU split (lab pg32lab, SDRG_CU_SPLIT=1).  GPU suite's SSB tests first.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssb_schedule.py tests/test_gpu_parity.py tests/test_gpu_ssb_variant.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pg32_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pg32_tests.log; exit 1; }
tail -1 gpurun_out/pg32_tests.log
L=$PWD/sdr-for-android-lib_amd/lib
run() {  # label lib split steps
  SDRG_LIB_PATH=$2 SDRG_CU_SPLIT=$3 timeout -k 10 200 python bench.py --steps $4 --warmup 5 --no-cpu-baseline --no-labelled > gpurun_out/pg32_$1.json 2> gpurun_out/pg32_$1.err || { echo "bench $1 failed"; tail -5 gpurun_out/pg32_$1.err; exit 1; }
  echo "$1 $(tail -1 gpurun_out/pg32_$1.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["ssb_latency_floor"]["ssb_ms_alone"], d["roofline_isolated"]["frac"])')"
}
run product "" "" 20
run pg16 $L/libsdrg_pg16.so "" 20
run mode1 $L/libsdrg_pg32lab.so 1 20
run product200 "" "" 200
run pg16_200 $L/libsdrg_pg16.so "" 200
run mode1_200 $L/libsdrg_pg32lab.so 1 200
