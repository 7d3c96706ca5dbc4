#!/bin/bash
# round 5 session 6: batch / pipeline / stagger correctness, colour prepd A/B, staggered round robin A/B at B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
F="--cpu-seconds 0.3 --no-latency --no-kernel-timing"
PYTEST_SECS=400 bash tools/gpu.sh r05_s6 tests="tests/test_gpu_parity.py::test_batch_equals_singles tests/test_gpu_configs.py" \
  bench_C="--config C --cpu-seconds 0.3 --no-latency" bench_C1="--config C --cpu-seconds 0.3 --no-latency --option prepd=1" \
  bench_B0="$F" bench_Bst="$F --option stagger=1" bench_Bst4="$F --option stagger=1 --chunk 1024" \
  bench_B3st="$F --option stagger=1 --streams 3 --chunk 1366" bench_B0b="$F"
