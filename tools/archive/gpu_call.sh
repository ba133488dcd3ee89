#!/bin/bash
# Run one gpurun call; if the box could not be prepared (status transient / exit 3: nothing ran, nothing
# charged) wait and try again, at most 6 times.  A call that ran is never repeated.
cmd="$1"; to="${2:-900}"
for attempt in 1 2 3 4 5 6; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > /tmp/gpu_call.out 2>&1
  rc=$?
  if grep -q "status=transient\|no box\|slot free" /tmp/gpu_call.out || [ $rc -eq 3 ]; then
    echo "attempt $attempt: transient, retrying" >&2; sleep 60; continue
  fi
  tail -3 /tmp/gpu_call.out; exit $rc
done
echo "gave up after transient failures" >&2; exit 3
