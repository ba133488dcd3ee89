#!/bin/bash
# round 4 HEAD check: full GPU suite, then the round profile (smoke, driver command, profile_round, SQ counters)
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r4c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
bash tools/gpu_r4_final.sh $TAG
