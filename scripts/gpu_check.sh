#!/usr/bin/env bash
# Run GPU validation steps on the gpurun box; each step has its own time limit and the
# script stops at the first step that ends by a signal / fault / timeout (anything other
# than success or an ordinary test failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
OUT="$PWD/gpurun_out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
step() {  # step <seconds> <logname> <cmd...>
  local secs=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do eval "$s" || exit $?; done
