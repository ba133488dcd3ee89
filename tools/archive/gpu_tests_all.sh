#!/bin/bash
# every -m gpu test in one process (per-test timeout), then smoke()
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc $rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/gpu_tests.log | tail -20; tail -5 gpurun_out/gpu_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -2
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
