#!/bin/bash
# Run one gpurun call, retrying ONLY while the pool answers "transient" (no box
# free, box lost while being prepared, back-off after an infrastructure
# failure: nothing of the command ran).  A call that ran -- passed or failed --
# is never repeated.  Usage: tools/gpu_retry.sh OUT_FILE TIMEOUT_S 'command'
set -u
out=$1; lim=$2; cmd=$3
for attempt in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient" "$out"; then
    echo "attempt $attempt: transient, waiting" >&2
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
