#!/bin/bash
# A/B runs of bench.py: each argument is one quoted option string, e.g. "--option nt_store=1".
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab}
mkdir -p "$OUT"
shift || true
k=0
for opts in "$@"; do
  k=$((k+1))
  echo "== [$k] $opts"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 $opts > "$OUT/r$k.json" 2> "$OUT/r$k.err"
  rc=$?
  python -c "import json; d=json.load(open('$OUT/r$k.json')); print(d['value'], d['ms_per_step'], {k:round(v['total_ms']/10,3) for k,v in d['kernels'].items()})" 2>/dev/null
  if [ $rc -ne 0 ]; then echo "stop rc=$rc"; tail -3 "$OUT/r$k.err"; exit $rc; fi
done
