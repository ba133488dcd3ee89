#!/bin/bash
# r5ai: HEAD check: smoke, the full GPU suite, the default bench line
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ai_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/r5ai_smoke.log; exit 1; }
tail -1 gpurun_out/r5ai_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5ai_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -30 gpurun_out/r5ai_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r5ai_gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r5ai_bench.json 2> gpurun_out/r5ai_bench.err || { tail gpurun_out/r5ai_bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r5ai_bench.json
