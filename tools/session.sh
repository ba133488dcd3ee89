#!/bin/bash
# r5am: the C-ABI gather test with its refusal cases
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dist_capi.py > gpurun_out/r5am_tests.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r5am_tests.log; exit 1; }
tail -1 gpurun_out/r5am_tests.log
