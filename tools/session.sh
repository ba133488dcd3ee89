#!/bin/bash
# r5ag: the C-ABI gather test over its three stream paths x two one-rank data paths
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist_capi.py > gpurun_out/r5ag_tests.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r5ag_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r5ag_tests.log; tail -1 gpurun_out/r5ag_tests.log
