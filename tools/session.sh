#!/bin/bash
# r5bj: SSB pipeline with two taps copies read as 8-byte pairs (lab SDRG_TAPS_COPIES=2, 3 KB less LDS): SSB tests on
# the lab build, then the c3 line and the SSB stage alone against the product, alternating
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh -r 2 -o r5bj -t "tests/test_gpu_parity.py tests/test_gpu_ssb_variant.py tests/test_gpu_ssb_schedule.py" base taps2 -- \
  python bench.py --no-cpu-baseline --no-labelled
