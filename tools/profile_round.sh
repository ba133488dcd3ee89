#!/bin/bash
# Round profile: bench line, rocprofv3 kernel-trace --stats of the same bench, and the two HBM PMC passes
# (FETCH_SIZE, WRITE_SIZE in separate runs, kernel-trace only) -> gpurun_out/*_$TAG; then
# tools/profile_summary.py $TAG writes profiles/.
export TMPDIR=/tmp
TAG=${1:-r1}
STEPS=${STEPS:-40}
# (the library is built in-tree on the CPU side before the call)
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
echo "bench: $(tail -1 gpurun_out/bench_$TAG.log | cut -c1-200)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup 50 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1 || { echo "rocprof stats failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmcf_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmcf_$TAG.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmcw_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmcw_$TAG.log 2>&1 || { echo "pmc write failed"; exit 1; }
echo "profile done"
