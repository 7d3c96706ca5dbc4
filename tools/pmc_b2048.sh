#!/bin/bash
# HBM traffic at the bench's own launch size (config B, 4096 pairs per step = two 2048-pair launches), one
# rocprofv3 --pmc pass per counter, counters only, restricted to the kernels the bench line's roofline fields
# read (tv_sor, upsample, aggregate, tv_system) so the pass stays short.  -> tools/pmc_traffic.py
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-pmc_b2048}
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c $(date +%T)"
  timeout -k 10 900 rocprofv3 --pmc $c --kernel-include-regex 'k_tv_sor|k_upsample|k_aggregate|k_tv_smsys|k_pyr_base' \
    -d "$OUT/$c" -o run --output-format csv -- \
    python -u bench.py --steps 1 --warmup 1 --no-kernel-timing --cpu-seconds 0 --no-latency --parity-frames 1 \
    > "$OUT/$c.log" 2>&1
  rc=$?
  echo "== pmc $c rc=$rc $(date +%T)"; tail -n 2 "$OUT/$c.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/pmc_traffic.py "$OUT/FETCH_SIZE" "$OUT/WRITE_SIZE" "1920x1080:op2:b2048" "$OUT/traffic.json"
