#!/bin/bash
# r5x: the full GPU suite at HEAD (gathers on the producing stream, statistics stream created with the engine)
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5x_tests.log 2>&1 || { echo "tests FAILED"; grep -E "FAILED|Error|error" gpurun_out/r5x_tests.log | head -20; tail -30 gpurun_out/r5x_tests.log; exit 1; }
tail -1 gpurun_out/r5x_tests.log
