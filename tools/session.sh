#!/bin/bash
# r5n: does a one-rank RCCL communicator or gloo group in the process slow kernels that run alone?
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for d in "" rccl gloo both; do
    SPEC_TIME_DIST=$d timeout -k 10 120 python tools/lab/spec_time.py 16384 cs8 4096 200 2>&1 | tail -1 || exit 1
  done
done
