#!/bin/bash
# r5aj: SSB pipeline role maps that take the equaliser off the low-pass wave's SIMD (lab SDRG_PIPE_MAP)
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh -r 2 -o map -t "tests/test_gpu_ssb_schedule.py" base lab:SDRG_PIPE_MAP=7B9846A53210 lab:SDRG_PIPE_MAP=7B984A563210 lab:SDRG_PIPE_MAP=7B986A453210 -- python bench.py --no-cpu-baseline --no-labelled
