#!/bin/bash
# PMC passes (each its own run, counters only) for one bench config: SQ stall/issue counters, FETCH_SIZE,
# WRITE_SIZE.  Usage: tools/pmc_config.sh OUTNAME CONFIG BATCH [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; CFG=$2; B=$3; shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python bench.py --config $CFG --batch $B --steps 1 --warmup 1 --distinct 2 --no-kernel-timing --cpu-seconds 0 --no-latency $*"
pass() {  # name counters...
  local name=$1; shift
  echo "== pmc $name: $*"; date
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 2 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
[ -f "$OUT/../counters.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$OUT/../counters.txt" 2>&1
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo "== done"
