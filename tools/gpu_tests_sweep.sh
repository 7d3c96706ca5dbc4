#!/bin/bash
# pytest -m gpu, then a (streams, chunk, graph) sweep of the default bench and the other configs' benches.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-tsweep}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== graph probe"; date
timeout -k 10 400 python tools/graph_probe.py > "$OUT/graph_probe.log" 2>&1
echo "graph probe rc=$?"; grep -E "^==|same|graph:|Fatal|Segm" "$OUT/graph_probe.log" | head -40
echo "== pytest"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout=300 --timeout-method=thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() {  # name, args...
  local name=$1; shift
  echo "== $name: $*"; date
  timeout -k 10 300 python bench.py --cpu-seconds 0 --no-latency "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  python -c "import json; d=json.load(open('$OUT/$name.json')); print(d['value'], d['ms_per_step'], {k:round(v['total_ms']/d['steps'],3) for k,v in d['kernels'].items()})" 2>/dev/null
  if [ $rc -ne 0 ]; then echo "stop rc=$rc"; tail -5 "$OUT/$name.err"; exit $rc; fi
}
run b_default --steps 10
run b_graph0 --steps 10 --option graph=0
run b_s4c256 --steps 10 --streams 4 --chunk 256
run b_s4c128 --steps 10 --streams 4 --chunk 128
run b_s8c128 --steps 10 --streams 8 --chunk 128
run b_s2c256 --steps 10 --streams 2 --chunk 256
run b_s4c128_nt --steps 10 --streams 4 --chunk 128 --option nt_store=1
run b_default_nt --steps 10 --option nt_store=1
run d_default --config D --steps 10
run c_default --config C --steps 3 --warmup 1
run c2_default --config C2 --steps 3 --warmup 1
run e_default --config E --steps 2 --warmup 1
echo "== done"
