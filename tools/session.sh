#!/bin/bash
# r5af: the spectrum's |X|^2 stores write-through (sc1) so that they leave no dirty L2 lines for the SSB kernel's
# end-of-kernel write-back (the ~6 us gap between consecutive SSB kernels), against nt (product) and plain
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh -r 2 -o st -t "tests/test_gpu_parity.py" base st16 st18 st0 -- python bench.py --no-cpu-baseline --no-labelled || exit 1
bash tools/ab.sh -r 2 -o std base st16 st18 -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-labelled
