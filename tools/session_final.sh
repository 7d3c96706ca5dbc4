set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02_s25
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout=300 --timeout-method=thread -p no:cacheprovider > gpurun_out/r02_s25/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r02_s25/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02_s25/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r02_s25/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r02_s25/bench.json 2> gpurun_out/r02_s25/bench.err; rc=$?; tail -c 400 gpurun_out/r02_s25/bench.json; exit $rc
