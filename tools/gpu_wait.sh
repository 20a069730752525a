#!/bin/bash
# gpurun with patient retries: only when no box was obtained (rc 3 / transient: nothing ran, nothing
# charged).  Usage: tools/gpu_wait.sh TIMEOUT ATTEMPTS 'command'
T=$1; N=$2; shift 2
for i in $(seq 1 "$N"); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  if [ $rc -eq 3 ] || echo "$out" | grep -q "status=transient"; then
    echo "[gpu_wait] transient (attempt $i), retrying in 120 s" >&2; sleep 120; continue
  fi
  echo "$out"; exit $rc
done
echo "$out"; exit $rc
