#!/bin/bash
# round 5 session 12: stream priorities in the pipeline (option prio); B lane layouts with the source-row upsample;
# D's 32-pair shard on 1 / 2 streams
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05_s12; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "batch_equals_singles" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--steps 10 --warmup 4 --cpu-seconds 0 --no-latency --parity-frames 2"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py $B "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "$n failed"; tail -3 $OUT/bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$n.json'));k=d.get('kernels',{});print('$n',d['value'],d['ms_per_step'],k.get('upsample',{}).get('avg_us'))"
}
run B_rr_up1 --config B
run B_rr_up0 --config B --option up_form=0
run B_s1 --config B --streams 1 --chunk 2048
run B_p1 --config B --option pipeline=1
run B_p1_pr1 --config B --option pipeline=1 --option prio=1
run B_p1_pr2 --config B --option pipeline=1 --option prio=2
run B_p2_pr1 --config B --option pipeline=2 --option prio=1
run B_p1_pr1_c1024 --config B --option pipeline=1 --option prio=1 --chunk 1024
run B_rr_up1b --config B
run D32_s1 --config D --total 32 --streams 1
run D32_s2c16 --config D --total 32 --streams 2 --chunk 16
run D32_p1c16 --config D --total 32 --option pipeline=1 --option prio=1 --chunk 16
run D32_s1b --config D --total 32 --streams 1
