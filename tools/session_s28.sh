#!/bin/bash
# run-to-run spread of the default bench: several timed regions inside one process, three processes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02_s28
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --no-latency --no-kernel-timing --cpu-seconds 0 --probe-regions 6 > gpurun_out/r02_s28/run$k.json 2> gpurun_out/r02_s28/run$k.err || exit 3
  grep "probe region" gpurun_out/r02_s28/run$k.err | tr '\n' ' '; python -c "import json; d=json.load(open('gpurun_out/r02_s28/run$k.json')); print('| reported', d['ms_per_step'])"
done
