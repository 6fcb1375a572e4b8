#!/bin/bash
# Round-4 GPU check: the whole GPU suite + smoke, then (optionally) the default bench line.
# Each GPU step has its own limit; a crash or timeout ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
K=${K:-}
case "${1:-test}" in
test)
  step pytest_gpu 900 python -u -m pytest tests -v -m gpu -rf --timeout 300 --timeout-method thread ${K:+-k "$K"}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  ;;
bench)
  step bench 600 python bench.py
  ;;
all)
  step pytest_gpu 900 python -u -m pytest tests -v -m gpu -rf --timeout 300 --timeout-method thread ${K:+-k "$K"}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step bench 600 python bench.py
  ;;
esac
echo "=== done"
