#!/bin/bash
# Round-6 HBM traffic per kernel for every bench config: two rocprofv3 --pmc passes each (FETCH_SIZE, WRITE_SIZE: they
# do not fit one pass on gfx950), counters only, each pass its own run under its own time limit, at the pairs per
# launch the bench config runs (bench.py config_tag).  Reduced by tools/pmc_traffic.py into gpurun_out/<out>/traffic.json
# (copied to profiles/traffic.json afterwards, every entry carrying its source).
#   tools/pmc_r05.sh <out> <config>:<batch>:<pairs-per-launch>[:<extra bench args, + for spaces>] ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:?out}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  IFS=: read -r CFG B PL EXTRA <<< "$spec"
  EXTRA=${EXTRA//+/ }
  TAG=$(python -c "import bench; print(bench.config_tag(bench.CONFIGS['$CFG'], $PL))")
  for c in FETCH_SIZE WRITE_SIZE; do
    D="$OUT/${CFG}_$c"
    echo "== $CFG $c ($TAG) $(date +%T)"
    # shellcheck disable=SC2086
    timeout -k 10 300 rocprofv3 --pmc $c -d "$D" -o run --output-format csv -- python bench.py --config "$CFG" \
      --batch "$B" --chunk "$PL" --streams 1 --steps 1 --warmup 1 --distinct 2 --no-kernel-timing --cpu-seconds 0 \
      --no-latency $EXTRA > "$D.log" 2>&1
    rc=$?
    echo "== rc=$rc"; tail -n 2 "$D.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
  python tools/pmc_traffic.py "$OUT/${CFG}_FETCH_SIZE" "$OUT/${CFG}_WRITE_SIZE" "$TAG" "$OUT/traffic.json" \
    "profiles/r06/pmc (round 6: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, $CFG at $PL pairs per launch)"
done
echo "== done $(date +%T)"
