#!/bin/bash
# r5au: NCO variant with the integer unpack scale folded into the phasors (LDS-DMA path): SSB tests, then A/B of
# the nco127 line against the previous lab build
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh -r 3 -o r5au -t "tests/test_gpu_ssb_variant.py tests/test_gpu_parity.py" labq labr -- \
  python bench.py --ssb-variant nco127 --no-cpu-baseline --no-labelled
