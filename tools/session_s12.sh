#!/bin/bash
# B's SOR / system issue + LDS counters, then the batch-size A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/pmc_sq2.sh r02_s12/pmc_B B 2048 || exit $?
bash tools/session_ab_opts.sh r02_s12/batch 20 "--no-kernel-timing --no-latency" "--batch 4096 --no-kernel-timing --no-latency" "--batch 3072 --no-kernel-timing --no-latency"
