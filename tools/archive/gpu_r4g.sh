#!/bin/bash
# round 4: the whole GPU suite + smoke on the product library, the wide-statistics variants (tools/gpu_r4f.sh), then the
# paired-stream FIR (SDRG_FIR_PAIRS) against the product pipeline (tools/gpu_ab_stamps.sh)
export TMPDIR=/tmp
bash tools/gpu_tests_all.sh || exit 1
bash tools/gpu_r4f.sh || exit 1
echo "== FIR pairs"
bash tools/gpu_ab_stamps.sh firp prodlab || exit 1
bash tools/gpu_r4h.sh
