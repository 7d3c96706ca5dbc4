#!/bin/bash
# One gpurun session, parameterised (replaces the round-2 one-off session_*.sh scripts).
#
#   tools/gpu.sh <out-name> <step> [<step> ...]
#
# steps (run in order; each under its own time limit; a fault / abort / timeout -- any exit other than 0 or
# 1 -- ends the session, and so does a failing test run):
#   smoke                      __graft_entry__.smoke()
#   tests[=<pytest args>]      pytest -m gpu (default: the whole tests/ directory), verbose, 120 s per test
#   bench[=<bench.py args>]    one bench.py line into <step-name>.json (repeatable: bench, bench2=..., ...)
#   rocprof[=<bench.py args>]  rocprofv3 --kernel-trace --stats over a short bench.py run
#   pmc=<counters>[@<bench.py args>]   one rocprofv3 --pmc pass (counters only, no traces)
#   cmd=<shell command>        anything else (e.g. a probe program), time limit 300 s
# Steps named with a suffix (bench_D=..., pmc_B2=...) keep their outputs apart.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:?out-name}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PYTEST_SECS=${PYTEST_SECS:-1500}

step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name (limit ${secs}s) $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}

for spec in "$@"; do
  name=${spec%%=*}
  arg=""
  [ "$name" != "$spec" ] && arg=${spec#*=}
  kind=${name%%_*}
  case "$kind" in
    smoke)
      step "$name" 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    tests)
      # shellcheck disable=SC2086
      step "$name" "$PYTEST_SECS" python -u -m pytest ${arg:-tests} -m gpu -v -x --timeout 120 \
        --timeout-method thread -p no:cacheprovider || exit 1 ;;
    bench*)
      # shellcheck disable=SC2086
      step "$name" 900 python -u bench.py $arg || exit 1
      grep '^{' "$OUT/$name.log" | tail -n 1 > "$OUT/$name.json" ;;
    rocprof*)
      # shellcheck disable=SC2086
      step "$name" 900 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- \
        python -u bench.py ${arg:---steps 5 --warmup 2 --cpu-seconds 0 --no-latency} || exit 1 ;;
    pmc*)
      counters=${arg%%@*}
      bargs="--steps 2 --warmup 1 --no-kernel-timing --cpu-seconds 0 --no-latency"
      [ "$counters" != "$arg" ] && bargs="$bargs ${arg#*@}"
      # shellcheck disable=SC2086
      step "$name" 600 rocprofv3 --pmc $counters -d "$OUT/$name" -o run --output-format csv -- \
        python -u bench.py $bargs || exit 1 ;;
    cmd*)
      step "$name" 300 bash -c "$arg" || exit 1 ;;
    *)
      echo "unknown step $spec"; exit 2 ;;
  esac
done
echo "== session done $(date +%T)"
