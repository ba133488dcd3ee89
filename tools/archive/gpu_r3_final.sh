#!/bin/bash
# Round-3 check at HEAD: the GPU suite, smoke, the driver's bench command, then the round profile (tools/profile_round.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r3c}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py --warmup 5 --steps 20 > gpurun_out/${TAG}_driverlike.json 2> gpurun_out/${TAG}_driverlike.err || { echo "bench failed"; tail gpurun_out/${TAG}_driverlike.err; exit 1; }
tail -1 gpurun_out/${TAG}_driverlike.json | cut -c1-300
bash tools/profile_round.sh $TAG
