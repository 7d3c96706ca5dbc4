#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pw1}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout=300 --timeout-method=thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for cfg in "B 10" "C 3" "C2 3" "E 2"; do
  set -- $cfg
  for w in ${WINDOWS:-1 0}; do
    timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup 1 --cpu-seconds 0 --no-latency --option patch_window=$w > $OUT/$1_w$w.json 2> $OUT/$1_w$w.err || { echo "bench $1 $w failed"; tail -3 $OUT/$1_w$w.err; exit 3; }
    python -c "import json; d=json.load(open('$OUT/$1_w$w.json')); k=d['kernels']; print('$1 w=$w', d['value'], d['ms_per_step'], 'patch ms/step', round(k['patch']['total_ms']/d['steps'],3), 'avg us', round(k['patch']['avg_us'],1))"
  done
done
