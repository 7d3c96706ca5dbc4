#!/bin/bash
# A/B timing of library builds: tools/ab_session.sh OUTNAME "CFG STEPS" ... -- LIB1 LIB2 ...
# Each config runs once per library, twice over in alternating order (ABBA), kernel timing on.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"
cfgs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done; shift
libs=("$@")
for cfg in "${cfgs[@]}"; do
  set -- $cfg
  for rep in 0 1; do
    order=("${libs[@]}"); if [ $rep -eq 1 ]; then order=($(printf '%s\n' "${libs[@]}" | tac)); fi
    for L in "${order[@]}"; do
      tag=$(basename "$L" .so)_$1_$rep
      OFDIS_LIB=$PWD/$L timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup 1 --cpu-seconds 0 --no-latency \
        > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { echo "bench $tag failed"; tail -3 "$OUT/$tag.err"; exit 3; }
      python -c "import json; d=json.load(open('$OUT/$tag.json')); k=d['kernels']; print('$tag', d['value'], d['ms_per_step'], 'patch ms/step', round(k['patch']['total_ms']/d['steps'],3))"
    done
  done
done
