#!/bin/bash
# gpurun wrapper: retries ONLY when no box was obtained (status=transient / rc 3: nothing ran,
# nothing charged).  Usage: tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient\|no box or slot free" || [ $rc -eq 3 ]; then
    echo "[gpu.sh] transient (attempt $i), retrying in 60 s" >&2; sleep 60; continue
  fi
  echo "$out"; exit $rc
done
echo "$out"; exit $rc
