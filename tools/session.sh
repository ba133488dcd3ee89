#!/bin/bash
# r5ax: the NCO variant's own SSB role map (product build): SSB tests, then the default bench line twice
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ssb_variant.py tests/test_gpu_parity.py tests/test_gpu_ssb_schedule.py > gpurun_out/r5ax_tests.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r5ax_tests.log; exit 1; }
tail -1 gpurun_out/r5ax_tests.log
for i in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r5ax_bench$i.json 2> gpurun_out/r5ax_bench$i.err || { tail gpurun_out/r5ax_bench$i.err; exit 1; }
  python tools/bench_summary.py gpurun_out/r5ax_bench$i.json
done
