#!/bin/bash
# round 5 session 8: the fused system + SOR launch at config A (60-row finest level: lanes nearly full), A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
F="--cpu-seconds 0.3"
bash tools/gpu.sh r05_s8 bench_A0="--config A $F" bench_A1="--config A $F --option sysor=1" \
  bench_A0b="--config A $F"
