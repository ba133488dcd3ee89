#!/bin/bash
# r5e: final HEAD check: smoke, GPU suite, the driver command and the default line
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
TAG=r5e
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_driverlike.json 2> gpurun_out/${TAG}_driverlike.err || { echo "bench failed"; tail gpurun_out/${TAG}_driverlike.err; exit 1; }
python tools/bench_summary.py gpurun_out/${TAG}_driverlike.json
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail gpurun_out/${TAG}_bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/${TAG}_bench.json
