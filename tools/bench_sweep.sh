#!/bin/bash
# Batch / stream sweep of bench.py on one GPU (each run under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-sweep}
mkdir -p "$OUT"
shift || true
for cfg in "$@"; do
  read -r B S C <<<"$(echo "$cfg" | tr ',' ' ')"
  echo "== batch=$B streams=$S chunk=$C"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch "$B" --streams "$S" --chunk "$C" --cpu-seconds 0 \
    --no-latency > "$OUT/b${B}_s${S}_c${C}.json" 2> "$OUT/b${B}_s${S}_c${C}.err"
  rc=$?
  python -c "import json,sys; d=json.load(open('$OUT/b${B}_s${S}_c${C}.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], {k:round(v['total_ms']/10,3) for k,v in d['kernels'].items()})" 2>/dev/null
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop rc=$rc"; exit $rc; fi
done
