#!/bin/bash
# round 5 session 13: colour march with filtered derivatives (smsys_deriv for RGB tall levels): parity, C / C2 A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05_s13; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -k "pipeline_bitexact or config_C or smsys_deriv or smsys_march or flat_regions" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--steps 4 --warmup 2 --cpu-seconds 0 --no-latency --parity-frames 2"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "$n failed"; tail -3 $OUT/bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$n.json'));k=d.get('kernels',{});print('$n',d['value'],d['ms_per_step'],{x:round(k[x]['total_ms']/d['steps'],2) for x in ('tv_prep','tv_system','patch') if x in k})"
}
run C_df1 --config C
run C_df0 --config C --option smsys_deriv=0
run C2_df1 --config C2
run C2_df0 --config C2 --option smsys_deriv=0
run C_df1b --config C
