#!/bin/bash
# round 5 session 9: SQ issue / wait counters of B's kernels (one 2048-pair launch per step), one pass
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05_s9; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES \
  -d $OUT/sq -o run --output-format csv -- python bench.py --batch 2048 --chunk 2048 --streams 1 --steps 1 --warmup 1 \
  --distinct 2 --no-kernel-timing --cpu-seconds 0 --no-latency > $OUT/sq.log 2>&1
echo "rc=$?"; tail -2 $OUT/sq.log
