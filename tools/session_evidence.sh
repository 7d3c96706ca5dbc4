#!/bin/bash
# Round evidence for the headline config: bench (driver's command), rocprofv3 kernel stats of the default and
# of the serialised launches, and the two PMC traffic passes.  Every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-evidence}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; date
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
step bench 600 python bench.py --steps 20 --warmup 5
step prof_default 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-latency --no-kernel-timing
step prof_serial 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-latency --no-kernel-timing --streams 1 --chunk 1024
BENCH_BATCH=2048 bash tools/pmc_session.sh ${1:-evidence}/pmc
