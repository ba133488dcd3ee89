#!/bin/bash
# CU split lab: the SSB stream and the spectrum/statistics stream on disjoint CU halves (SDRG_CU_SPLIT), with the
# SSB pipeline's raw-IQ batches shrunk to 256 B per stream (variant raw256: 76 KiB LDS, two workgroups per CU).
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/sdr-for-android-lib_amd/lib/libsdrg_raw256.so
SDRG_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ssb or pipelined or full_size" > gpurun_out/split_parity.log 2>&1 || { echo "parity failed"; tail -20 gpurun_out/split_parity.log; exit 1; }
tail -1 gpurun_out/split_parity.log
run() {  # label lib split
  SDRG_LIB_PATH=$2 SDRG_CU_SPLIT=$3 timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-labelled > gpurun_out/split_$1.log 2>&1 || { echo "bench $1 failed"; tail -5 gpurun_out/split_$1.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/split_$1.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernel_ms"], d["ssb_latency_floor"]["ssb_ms_alone"], d["roofline_isolated"]["frac"])')"
}
run default "" 0
run raw256 $V 0
run split1 $V 1
run split2 $V 2
run default_b "" 0
run split1_b $V 1
