#!/bin/bash
# HBM traffic per kernel: two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE do not fit one pass on gfx950),
# each its own run, counters only.  Then tools/pmc_traffic.py -> profiles/traffic.json.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pmc}
B=${BENCH_BATCH:-1024}
C=$(( B >= 512 ? (B + 1) / 2 : B ))  # pairs per launch: bench.py / the library split >= 512 pairs over 2 streams
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c"; date
  timeout -k 10 600 rocprofv3 --pmc $c -d "$OUT/$c" -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --batch "$B" --no-kernel-timing --cpu-seconds 0 --no-latency > "$OUT/$c.log" 2>&1
  rc=$?
  echo "== pmc $c rc=$rc"; tail -n 3 "$OUT/$c.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/pmc_traffic.py "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE" "1920x1080:op2:b$C" "$OUT/traffic.json"
