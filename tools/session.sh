#!/bin/bash
# r5g: HEAD check after the lab-only statistics options (product code path unchanged): smoke, GPU suite, driver command
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
TAG=r5g
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_driverlike.json 2> gpurun_out/${TAG}_driverlike.err || { echo "bench failed"; tail gpurun_out/${TAG}_driverlike.err; exit 1; }
python tools/bench_summary.py gpurun_out/${TAG}_driverlike.json
