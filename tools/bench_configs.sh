#!/bin/bash
# All BASELINE configs through bench.py on one GPU (each run under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-configs}
mkdir -p "$OUT"
shift || true
for c in "$@"; do
  echo "== config $c"
  case $c in C|C2|E) extra="--parity-frames 2 --distinct 2";; *) extra="";; esac
  timeout -k 10 500 python bench.py --config "$c" --steps 5 --warmup 2 --cpu-seconds 15 --host-io $extra \
    > "$OUT/$c.json" 2> "$OUT/$c.err"
  rc=$?
  python -c "import json; d=json.load(open('$OUT/$c.json')); print(d['config']['workload'], d['value'], d['ms_per_step'], d['parity'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None, d['host_io'], d['roofline']['kernel'], d['roofline']['frac'])" 2>/dev/null
  if [ $rc -ne 0 ]; then echo "stop rc=$rc"; tail -5 "$OUT/$c.err"; exit $rc; fi
done
