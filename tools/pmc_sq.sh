#!/bin/bash
# SQ stall breakdown per kernel (one PMC pass, counters only).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pmc_sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES \
  -d "$OUT/sq" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-kernel-timing --cpu-seconds 0 --batch ${BENCH_BATCH:-0} > "$OUT/sq.log" 2>&1
echo "rc=$?"
