#!/bin/bash
# standard GPU round: build, gpu tests, bench, rocprof kernel trace (outputs under gpurun_out/)
export TMPDIR=/tmp
TAG=${1:-x}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 500 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; echo "pytest exit $?" >> gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo "prof exit $?"
