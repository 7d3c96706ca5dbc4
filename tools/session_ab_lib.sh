#!/bin/bash
# GPU tests of the tree's library, then an ABBA timing of library builds (tools/ab_session.sh).
# Usage: tools/session_ab_lib.sh OUTNAME "CFG STEPS" ... -- LIB1 LIB2 ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout=300 --timeout-method=thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
bash tools/ab_session.sh "$@"
