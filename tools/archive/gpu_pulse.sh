#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pulse.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_pulse.log 2>&1; rc=$?
echo "pytest rc $rc" >> gpurun_out/gpu_pulse.log
tail -25 gpurun_out/gpu_pulse.log
exit $rc
