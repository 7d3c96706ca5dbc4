#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/session_ab_lib.sh r02_s13 "B 10" "A 10" "D 10" -- ablib/libofdis_head.so ablib/libofdis_dpt.so || exit $?
bash tools/pmc_sq2.sh r02_s13/pmc_B B 2048 || exit $?
OFDIS_LIB=$PWD/ablib/libofdis_head.so bash tools/pmc_sq2.sh r02_s13/pmc_B_head B 2048 || exit $?
