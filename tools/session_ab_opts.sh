#!/bin/bash
# ABBA timing of option strings on the tree's library: tools/session_ab_opts.sh OUT STEPS "opts A" "opts B" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; STEPS=$2; shift 2; mkdir -p "$OUT"
for rep in 0 1; do
  k=0
  list=("$@"); if [ $rep -eq 1 ]; then list=(); for ((i=$#; i>0; i--)); do list+=("${!i}"); done; fi
  for o in "${list[@]}"; do
    tag=$(echo "$o" | tr -c 'A-Za-z0-9=_' '_')_$rep
    timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --cpu-seconds 0 $o > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { echo "fail $tag"; tail -3 "$OUT/$tag.err"; exit 3; }
    python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['ms_per_step'], {k:round(v['total_ms']/d['steps'],3) for k,v in d['kernels'].items() if k in ('tv_sor','tv_system')}, (d.get('latency') or {}).get('device_ms_median'))"
  done
done
