set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02_s6; mkdir -p $OUT
run() { tag=$1; lib=$2; shift 2
  OFDIS_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-latency "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { echo "fail $tag"; tail -3 $OUT/$tag.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['ms_per_step'], {k:round(v['total_ms']/d['steps'],1) for k,v in d['kernels'].items() if k in ('tv_system','tv_sor','patch')})"; }
for rep in 0 1; do
  run base_E_$rep ablib/libofdis_base.so --config E
  run mask_E_$rep ablib/libofdis_mask2d.so --config E --option smsys2d=0
  run m2d_E_$rep ablib/libofdis_mask2d.so --config E
  run m2d_s1_E_$rep ablib/libofdis_mask2d.so --config E --streams 1 --chunk 512
  run base_s1_E_$rep ablib/libofdis_base.so --config E --streams 1 --chunk 512
done
