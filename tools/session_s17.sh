#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02_s17
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "variants" --timeout=300 --timeout-method=thread -p no:cacheprovider > gpurun_out/r02_s17/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r02_s17/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/session_ab_opts.sh r02_s17/ab 10 "--no-latency" "--option nt_store=2 --no-latency" "--option nt_store=3 --no-latency"
