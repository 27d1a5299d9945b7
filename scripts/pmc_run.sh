#!/usr/bin/env bash
# One rocprofv3 PMC pass per counter file, summarised per kernel (CSV output, kernel filter).
#   bash scripts/pmc_run.sh <regex> <out_dir> <counter_file>... -- <program args...>
# Each pass runs under its own 90 s kill-timeout; the summary goes to <out_dir>/<name>.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
regex=$1; out=$2; shift 2
files=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do files+=("$1"); shift; done
shift
mkdir -p "$out"
for f in "${files[@]}"; do
  name=$(basename "$f" .txt)
  d=/tmp/pmc_$name_$$
  timeout -s KILL 90 rocprofv3 -i "$f" --kernel-include-regex "$regex" --output-format csv \
      -d "$d" -o run -- "$@" > "$out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee "$out/$name.txt"
  python3 scripts/pmc_summary.py "$d" | tee -a "$out/$name.txt"
  rm -rf "$d"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
