#!/bin/bash
# SQ issue / wait counters of the latency-mode single pair (tools/latency_calls.py, sor_mode = 1), two passes
# (counters only, each its own run and time limit): the per-wave cycle / wait / issue breakdown of k_tv_level_rb.
#   tools/sq_latency.sh <out>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:?out}; mkdir -p "$OUT"; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"
P2="SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
n=0
for P in "$P1" "$P2"; do
  n=$((n + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/sq$n" -o run --output-format csv -- python tools/latency_calls.py \
    --reps 5 --option sor_mode=1 > "$OUT/sq$n.log" 2>&1
  rc=$?; echo "pass $n rc=$rc"; tail -2 "$OUT/sq$n.log"
  [ $rc -eq 0 ] || exit $rc
done
