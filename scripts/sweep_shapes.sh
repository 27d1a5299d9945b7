#!/usr/bin/env bash
# Lloyd step throughput over (D, K) on one GPU, N=10M points, bf16 (bench.py); one JSON
# line per shape into gpurun_out/shapes.jsonl.  Each run under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
out=gpurun_out/shapes.jsonl
: > "$out"
for d in 64 128 256; do
  for k in 256 1024 4096 16384; do
    timeout -k 10 120 python -u bench.py --dim "$d" --k "$k" --steps 10 --warmup 2 > gpurun_out/_s.log 2>&1 || exit $?
    tail -1 gpurun_out/_s.log >> "$out"
    echo "d=$d k=$k done"
  done
done
