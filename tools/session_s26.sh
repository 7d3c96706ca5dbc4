#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/session_ab_opts.sh r02_s26/ab 10 "--no-latency --cpu-seconds 1 --parity-frames 4" "--option sor_rows2=2 --no-latency --cpu-seconds 1 --parity-frames 4" "--config A --option sor_rows2=2 --no-latency --cpu-seconds 1 --parity-frames 4" "--config A --no-latency --cpu-seconds 1 --parity-frames 4"
