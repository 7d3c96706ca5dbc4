#!/bin/bash
# Round evidence in one GPU call: GPU tests, the headline bench (driver's command), rocprofv3 kernel stats of
# the default and the serialised launches, PMC traffic for B, all BASELINE configs, PMC traffic for C and E.
# Every GPU step has its own time limit; the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-round}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name"; date
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 $OUT/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -x --timeout=300 --timeout-method=thread -p no:cacheprovider
step bench 600 python bench.py --steps 20 --warmup 5
cp $OUT/bench.log $OUT/bench_default.json
step prof_default 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-latency --no-kernel-timing
step prof_serial 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-latency --no-kernel-timing --streams 1 --chunk 1024
BENCH_BATCH=2048 bash tools/pmc_session.sh ${1:-round}/pmc_B || exit $?
bash tools/bench_configs.sh ${1:-round}/configs A C C2 D E || exit $?
bash tools/pmc_config.sh ${1:-round}/pmc_C C 512 || exit $?
bash tools/pmc_config.sh ${1:-round}/pmc_E E 512 || exit $?
bash tools/pmc_sq2.sh ${1:-round}/pmc_Bsq B 2048 || exit $?
echo "== session done"
