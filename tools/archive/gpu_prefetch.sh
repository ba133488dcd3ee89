#!/bin/bash
# SSB raw-IQ prefetch depth under co-residency: default (512 B x 2 batches: 4 chunks ahead), nraw3/nraw4 (256 B x 3/4:
# 4/6 chunks ahead, same or less LDS); parity of the variants, bench lines, and the in-kernel clock (stamps)
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in nraw4 nraw3; do
  SDRG_LIB_PATH=$PWD/sdr-for-android-lib_amd/lib/libsdrg_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine_api.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ssb or pipelined or full_size or batch" > gpurun_out/pf_parity_$v.log 2>&1 || { echo "parity $v failed"; tail -20 gpurun_out/pf_parity_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/pf_parity_$v.log)"
done
run() {  # label lib
  SDRG_LIB_PATH=$2 timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-labelled > gpurun_out/pf_$1.log 2>&1 || { echo "bench $1 failed"; tail -5 gpurun_out/pf_$1.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/pf_$1.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["ssb_latency_floor"]["ssb_ms_alone"])')"
}
L=$PWD/sdr-for-android-lib_amd/lib
run default ""
run nraw4 $L/libsdrg_nraw4.so
run nraw3 $L/libsdrg_nraw3.so
run default_b ""
run nraw4_b $L/libsdrg_nraw4.so
# clocks: stamps of the last timed (co-resident) call and of the last SSB-alone call
SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-labelled > gpurun_out/pf_stamps.log 2>&1 || { echo "stamps failed"; exit 1; }
grep "LPF\|LOAD" gpurun_out/pf_stamps.log
