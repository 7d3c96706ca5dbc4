#!/bin/bash
# Runs tools/bin/capture_repro (built from tools/capture_repro.hip) mode by mode; stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-capture}; mkdir -p "$OUT"
for m in ${MODES:-0 1 3 2 5 4}; do
  echo "== mode $m"
  timeout -k 10 60 tools/bin/capture_repro $m 3 > "$OUT/mode$m.log" 2>&1
  rc=$?
  cat "$OUT/mode$m.log"; echo "rc=$rc"
  if [ $rc -ne 0 ]; then echo "stopping after mode $m"; exit 0; fi
done
