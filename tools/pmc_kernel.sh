#!/bin/bash
# Issue counters of the kernels matching a regex in one bench config (two SQ passes, each its own run):
#   tools/pmc_kernel.sh OUTNAME CONFIG BATCH REGEX [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; CFG=$2; B=$3; RX=$4; shift 4
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python bench.py --config $CFG --batch $B --steps 1 --warmup 1 --distinct 2 --no-kernel-timing --cpu-seconds 0 --no-latency $*"
pass() {
  local name=$1; shift
  echo "== pmc $name: $*"; date
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
pass sqa SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
pass sqb SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_VMEM
echo "== done"
