#!/usr/bin/env bash
# The reference's own sweep (scripts/new_experiment.py grid: N in {100M, 75M, 50M, 25M}, D=5,
# K in {15, 12, 9, 6, 3}, both methods, 20 iterations, make_classification data, seed
# 1826273) through the compatible entry points, in fp64 (the reference's dtype) and fp32,
# on every GPU count this node has (1..8; counts above the node's are skipped), one
# rocprofv3 trace per run -- the like-for-like of scripts/executions_log.csv.
#
#   scripts/like_for_like.sh OUTDIR [GPU counts...]      (default: 1 2 3 4 5 6 7 8)
#   DTYPES=fp32 scripts/like_for_like.sh OUTDIR 1         (one dtype pass only)
#
# --no_warmup: the reference's computation_time includes its first sess.run.  Re-runnable:
# --skip_done keeps the rows already in the logs.  Compile and compare afterwards with
#   python scripts/compileResults.py --input_dir OUTDIR/rocprof_fp64 --output_dir OUTDIR/compiled_fp64
#   python scripts/compare_with_reference.py --ours fp64=OUTDIR/executions_log_mi355x_fp64.csv \
#       --ours fp32=OUTDIR/executions_log_mi355x_fp32.csv --reference <ref>/scripts/executions_log.csv
set -o pipefail
OUT=${1:-results/like_for_like}
shift || true
GPUS=${*:-1 2 3 4 5 6 7 8}
mkdir -p "$OUT"
for DT in ${DTYPES:-fp64 fp32}; do
  python scripts/new_experiment.py --gpus $GPUS --skip_unavailable --skip_done \
      --log_file "$OUT/executions_log_mi355x_$DT.csv" --log_dir "$OUT/rocprof_$DT" \
      --data_file "${TMPDIR:-/tmp}/class-data.npz" --timeout 900 -- --dtype "$DT" --no_warmup \
      || exit $?
done
