#!/bin/bash
# One gpurun session: smoke -> pytest -m gpu -> short bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; any fault/abort/timeout (exit not in {0,1}) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name (limit ${secs}s)"; date
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -x --timeout=300 --timeout-method=thread -p no:cacheprovider
step bench 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 3 --batch ${BENCH_BATCH:-0}
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --batch ${BENCH_BATCH:-0} --cpu-seconds 0 --no-latency
fi
echo "== session done"
