#!/bin/bash
# GPU tests, then default vs red-black SOR benches for B and D (with the single-pair latency leg and a short
# parity sample against the oracle).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-rb1}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout=300 --timeout-method=thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest_gpu.log"; grep "red-black vs exact" "$OUT/pytest_gpu.log" | head
grep -o "red-black vs exact.*" "$OUT/pytest_gpu.log" | head
if [ $rc -ne 0 ]; then exit $rc; fi
for cfg in "B 10" "D 20"; do
  set -- $cfg
  for m in 0 1; do
    timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup 3 --cpu-seconds 0.5 --option sor_mode=$m > $OUT/$1_m$m.json 2> $OUT/$1_m$m.err || { echo "bench $1 $m failed"; tail -3 $OUT/$1_m$m.err; exit 3; }
    python -c "import json; d=json.load(open('$OUT/$1_m$m.json')); k=d['kernels']; print('$1 sor_mode=$m', d['value'], d['ms_per_step'], 'sor ms/step', round(k['tv_sor']['total_ms']/d['steps'],3), 'parity', d['parity'], 'latency ms', d['latency']['device_ms_median'], d['latency']['host_ms_median'])"
  done
done
