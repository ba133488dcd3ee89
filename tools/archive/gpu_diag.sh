#!/bin/bash
# stage ablations + SSB pipeline stamps (diagnostic)
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
for st in spectrum spectrum+stats ssb all; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --stages $st > gpurun_out/abl_$st.log 2>&1 || { echo "abl $st failed"; exit 1; }
done
SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/stamps.log 2>&1
echo "stamps exit $?"
