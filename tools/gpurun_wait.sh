#!/bin/bash
# gpurun with waiting for a free slot: retries ONLY when gpurun reports that no slot / box was free
# (nothing ran, nothing charged); any call that ran -- whatever its outcome -- is never repeated.
#   tools/gpurun_wait.sh <log> <timeout-s> '<command>'
LOG=${1:?log}; TMO=${2:?timeout}; CMD=${3:?command}
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && grep -q -E "nothing was charged|not charged" "$LOG"; then
    echo "attempt $i: no slot, waiting" >> "$LOG.wait"
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
