#!/bin/bash
# r5at: integer-format unpack scale on sample pairs (packed) in the SSB loaders: SSB tests, then A/B of the nco127
# and the c3 lines against the previous lab build
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh -r 3 -o r5at_nco -t "tests/test_gpu_ssb_variant.py tests/test_gpu_parity.py tests/test_gpu_ssb_schedule.py" labp labq -- \
  python bench.py --ssb-variant nco127 --no-cpu-baseline --no-labelled &&
bash tools/ab.sh -r 2 -o r5at_c3 labp labq -- python bench.py --no-cpu-baseline --no-labelled
