#!/bin/bash
# Run one gpurun call, retrying only while the pool has no free box (exit 3:
# nothing ran, nothing charged), at most TRIES times, SLEEP seconds apart.
#   tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; tmo=$2; cmd=$3
TRIES=${TRIES:-12}; SLEEP=${SLEEP:-150}
for i in $(seq 1 $TRIES); do
  /usr/local/graft/bin/gpurun --timeout "$tmo" -- "$cmd" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && ! grep -q "status=transient" "$out" && exit $rc
  echo "[retry $i: no box]" >> "$out.retries"
  sleep $SLEEP
done
exit 3
