#!/bin/bash
# round 5 session 5: full GPU suite (colour prepd now default), C / C2 / E benches with A/B of the colour prepd,
# then the PMC traffic passes of every config (tools/pmc_r05.sh)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PYTEST_SECS=600 bash tools/gpu.sh r05_s5 smoke tests bench_C="--config C --cpu-seconds 0.5 --no-latency" \
  bench_C1="--config C --cpu-seconds 0.5 --no-latency --option prepd=1" bench_C2="--config C2 --cpu-seconds 0.5 --no-latency" \
  bench_E="--config E --cpu-seconds 0.5 --no-latency" || exit $?
bash tools/pmc_r05.sh r05_s5/pmc B:2048:2048 A:1024:1024 D:256:256 C:256:256 C2:256:256 E:256:256
