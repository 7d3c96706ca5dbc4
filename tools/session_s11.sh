#!/bin/bash
# round 5 session 11: parity of the fast pivot division (patch_fdiv), the largest-|w| stopping test (patch_maxres)
# and the source-row upsample (up_form); then A/B bench lines: B with up_form 0/1/2, E and C with both patch
# options on / off
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05_s11; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "flat_regions or upsample_forms or patch_fdiv or patch_maxres or up_form or full_1080p or pipeline_bitexact" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="--steps 10 --warmup 4 --cpu-seconds 0 --no-latency"
for f in 1 0 2; do
  timeout -k 10 300 python bench.py --config B $B --option up_form=$f > $OUT/bench_B_up$f.json 2> $OUT/bench_B_up$f.err || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_B_up$f.json'));print('B up_form=$f',d['value'],d['kernels']['upsample']['avg_us'],d['kernels']['patch']['avg_us'])"
done
for cfg in E C; do
  for v in "1 1" "0 0" "1 0"; do
    set -- $v
    timeout -k 10 400 python bench.py --config $cfg --steps 3 --warmup 2 --cpu-seconds 0 --no-latency --option patch_fdiv=$1 \
      --option patch_maxres=$2 > $OUT/bench_${cfg}_fd$1mr$2.json 2> $OUT/bench_${cfg}_fd$1mr$2.err || exit 1
    python -c "import json;d=json.load(open('$OUT/bench_${cfg}_fd$1mr$2.json'));print('$cfg fdiv=$1 maxres=$2',d['value'],d['kernels']['patch']['avg_us'])"
  done
done
