#!/bin/bash
# Round 3: wide-statistics full-EXEC A/B, then the instruction-cache counters available on gfx950 and their values for
# the wide statistics kernel, then the SQ counter passes at HEAD (tools/gpu_sq_profile.sh, tag r3d).
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_wide_fe.sh || exit 1
cd /tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1; cd $GRAFT_REPO_ROOT
grep -i -o "SQC_[A-Z0-9_]*\|SQ_IFETCH[A-Z0-9_]*\|SQ_WAIT_INST_ANY\|SQ_INST_LEVEL[A-Z_]*" gpurun_out/counters_list.txt | sort -u | tr '\n' ' '; echo
PROGS="spec c2 c5 c3 ssb" bash tools/gpu_sq_profile.sh r3d || exit 1
