#!/bin/bash
# One A/B runner for every lab comparison (replaces round 4's per-experiment scripts, now in tools/archive/).
#
#   tools/ab.sh [-r ROUNDS] [-t "TEST_FILES"] [-o TAG] VARIANT... -- COMMAND...
#
# VARIANT: "base" (the product library, sdr-for-android-lib_amd/lib/libsdrg.so) or NAME for a lab build made here by
# tools/build_variant.sh NAME "FLAGS" (lib/libsdrg_NAME.so), optionally with lab environment knobs as
# NAME:KEY=VAL,KEY=VAL (lab builds only read them); NAME+TAG runs build NAME under the label NAME+TAG (one build,
# several knob settings).  For each round the variants run COMMAND in turn (alternating,
# one box), each under its own time limit; a COMMAND that prints a bench.py JSON line is summarised (value, ms/step,
# per-kernel ms, labelled lines), anything else is shown as its last line.  -t: the listed GPU tests run once per
# non-base variant first (bit-exactness before timing).  Outputs under gpurun_out/ab_TAG_*.
# Example:  tools/ab.sh -r 3 base lpf64 -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled
set -o pipefail
export TMPDIR=/tmp
ROUNDS=2; TESTS=""; TAG=ab
while getopts "r:t:o:" opt; do
  case $opt in r) ROUNDS=$OPTARG ;; t) TESTS=$OPTARG ;; o) TAG=$OPTARG ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
[ ${#VARS[@]} -gt 0 ] && [ $# -gt 0 ] || { echo "usage: tools/ab.sh [-r N] [-t TESTS] [-o TAG] VARIANT... -- COMMAND..."; exit 2; }
D=sdr-for-android-lib_amd/lib
mkdir -p gpurun_out

run_env() {  # $1 = VARIANT spec: prints "KEY=VAL ..." for env
  local name=${1%%:*} knobs=""
  [ "$1" != "$name" ] && knobs=${1#*:}
  local libname=${name%%+*} lib=$D/libsdrg.so  # NAME+TAG: the build NAME under another label (other knobs)
  [ "$libname" != "base" ] && lib=$D/libsdrg_$libname.so
  # knobs are split at commas that start a new KEY= (so a value may hold commas: SDRG_STREAM_PRIO=0,-1)
  echo "SDRG_LIB_PATH=$lib $(echo "$knobs" | sed 's/,\([A-Z_][A-Z0-9_]*=\)/ \1/g')"
}

summarise() {
  python3 - "$1" <<'EOF'
import json, sys
lines = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')]
if not lines:
    print("  (no bench line)")
    sys.exit(0)
d = json.loads(lines[-1])
k = d.get("kernel_ms", {})
s = f"  {d['value'] / 1e3:.1f} G  {d['ms_per_step']:.4f} ms/step  spec {k.get('spectrum_ms', 0):.4f} stats {k.get('stats_ms', 0):.4f} ssb {k.get('ssb_ms', 0):.4f}"
fl = d.get("ssb_latency_floor")
if fl:
    s += f"  ssb_alone {fl['ssb_ms_alone']:.4f}"
print(s)
for name, l in d.get("labelled", {}).items():
    print(f"    {name}: {l['value'] / 1e3:.1f} G {l['ms_per_step']} ms" + (f" spec {l['spectrum_ms']} stats {l['stats_ms']}" if 'stats_ms' in l else ""))
EOF
}

if [ -n "$TESTS" ]; then
  for v in "${VARS[@]}"; do
    [ "${v%%[:+]*}" == "base" ] && continue
    env $(run_env "$v") timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS \
      > gpurun_out/ab_${TAG}_tests_${v%%:*}.log 2>&1 || { echo "tests FAILED on $v"; tail -30 gpurun_out/ab_${TAG}_tests_${v%%:*}.log; exit 1; }
    echo "tests on $v: $(tail -1 gpurun_out/ab_${TAG}_tests_${v%%:*}.log)"
  done
fi
for r in $(seq 1 $ROUNDS); do
  for v in "${VARS[@]}"; do
    out=gpurun_out/ab_${TAG}_${r}_${v%%:*}.log
    env $(run_env "$v") timeout -k 10 400 "$@" > $out 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "round $r $v: exit $rc"; tail -20 $out; exit 1; fi
    echo "round $r $v:"
    if grep -q '"metric"' $out; then summarise $out; else echo "  $(tail -1 $out)"; fi
  done
done
