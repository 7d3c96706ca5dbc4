#!/bin/bash
# round 5 session 14: four-lane patches reading each bilinear tap once per window row (patch_qrows): parity, E / B / D A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05_s14; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -k "pipeline_bitexact or patch_ or flat_regions or config_E or full_1080p or config_D or config_A" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--steps 4 --warmup 2 --cpu-seconds 0 --no-latency --parity-frames 2"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "$n failed"; tail -3 $OUT/bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$n.json'));k=d.get('kernels',{});print('$n',d['value'],d['ms_per_step'],{x:round(k[x]['total_ms']/d['steps'],2) for x in ('patch','tv_system','tv_sor','upsample') if x in k})"
}
run E_qr1 --config E
run E_qr0 --config E --option patch_qrows=0
run B_qr1 --config B --steps 10 --warmup 4
run B_qr0 --config B --steps 10 --warmup 4 --option patch_qrows=0
run D32_qr1 --config D --total 32 --streams 1 --steps 20 --warmup 5
run D32_qr0 --config D --total 32 --streams 1 --steps 20 --warmup 5 --option patch_qrows=0
run E_qr1b --config E
