#!/bin/bash
# r5ak: lab-knob test with the round-5 knobs, C-ABI tests
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lab_knobs.py tests/test_gpu_engine_api.py > gpurun_out/r5ak_tests.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r5ak_tests.log; exit 1; }
tail -1 gpurun_out/r5ak_tests.log
