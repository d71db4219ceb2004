#!/bin/bash
# Run one gpurun call, re-submitting it only while the pool has no box for it (gpurun's exit 3 / "transient":
# nothing ran, nothing was charged); any other outcome -- success, a failed or killed GPU step -- ends it.
#   bash tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$OUT"; then exit $rc; fi
  sleep 150
done
exit 3
