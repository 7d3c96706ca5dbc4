#!/bin/bash
# GPU parity suite, then an A/B of library builds: tools/gpu_parity_ab.sh OUTNAME "CFG STEPS" ... -- LIB...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout=300 --timeout-method=thread -p no:cacheprovider > gpurun_out/$1/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/$1/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab_session.sh "$@"
