#!/bin/bash
# round 5 session 7: the half-split SOR (sor_half) -- parity, then A/B at B, D and A
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
F="--cpu-seconds 0.3 --no-latency"
PYTEST_SECS=400 bash tools/gpu.sh r05_s7 tests="tests/test_gpu_sysor.py -k half" \
  bench_B0="$F" bench_B1="$F --option sor_half=1" bench_D0="--config D --cpu-seconds 0" \
  bench_D1="--config D --cpu-seconds 0 --option sor_half=1" bench_A0="--config A $F" bench_A1="--config A $F --option sor_half=1"
