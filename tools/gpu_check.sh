#!/bin/bash
# quick GPU validation: gpu tests (per-test timeout), fftlab, one bench line
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc $rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 5 120 ./tools/fftlab/fftlab > gpurun_out/fftlab.log 2>&1 || { echo fftlab failed; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench.log; exit 1; }
echo ok
