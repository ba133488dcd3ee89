#!/bin/bash
# r5as: NCO variant mix on sample pairs (packed products, planar phasors): variant tests, then A/B of the nco127
# line against the previous lab build
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh -r 3 -o r5as -t "tests/test_gpu_ssb_variant.py" lab labp -- \
  python bench.py --ssb-variant nco127 --no-cpu-baseline --no-labelled
