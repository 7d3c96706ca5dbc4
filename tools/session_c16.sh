set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout=300 -k "config_C or 192-128-3 or 96-64" > gpurun_out/c16_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/c16_pytest.log; [ $rc -eq 0 ] || exit $rc
for w in 1 3 2 0; do timeout -k 10 300 python bench.py --config C --steps 3 --warmup 1 --cpu-seconds 0 --no-latency --option patch_window=$w > gpurun_out/c16_w$w.json || exit 3; python -c "import json; d=json.load(open('gpurun_out/c16_w$w.json')); print($w, d['value'], d['kernels']['patch']['total_ms']/d['steps'])"; done
