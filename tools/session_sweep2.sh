#!/bin/bash
# B-config bench sweep: chunking / streams / pipeline (each its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-sweep2}; shift; mkdir -p $OUT
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-latency $args > $OUT/run$i.json 2> $OUT/run$i.err || { echo "run $i failed: $args"; tail -3 $OUT/run$i.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/run$i.json')); print('$args |', d['value'], d['ms_per_step'])"
done
