#!/bin/bash
# Round check at HEAD (tools/gpu_round_final.sh TAG): smoke, the driver's bench command, the round profile (tools/profile_round.sh: bench line,
# rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes), then SQ counters of the c5 and c3 programs
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r6x}
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python bench.py --warmup 5 --steps 20 > gpurun_out/${TAG}_driverlike.json 2> gpurun_out/${TAG}_driverlike.err || { echo "bench failed"; tail gpurun_out/${TAG}_driverlike.err; exit 1; }
tail -1 gpurun_out/${TAG}_driverlike.json | cut -c1-200
bash tools/profile_round.sh $TAG || exit 1
PROGS="c5 c3" bash tools/gpu_sq_profile.sh ${TAG}sq || exit 1
