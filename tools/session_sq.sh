#!/bin/bash
# round 5 session 10: SQ issue / wait counters of E's and C's kernels (one 256-pair launch), one pass each
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r05_s10}; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in E C; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES \
    -d $OUT/sq_$cfg -o run --output-format csv -- python bench.py --config $cfg --batch 256 --chunk 256 --streams 1 --steps 1 --warmup 1 \
    --distinct 2 --no-kernel-timing --cpu-seconds 0 --no-latency > $OUT/sq_$cfg.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; tail -2 $OUT/sq_$cfg.log
  [ $rc -eq 0 ] || exit $rc
done
