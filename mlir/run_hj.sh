#!/bin/bash
# run_hj.sh <file.mlir> -- the reference's run_test.sh pipeline (run_test.sh:
# 21-33) with libhj.so on --shared-libs.  The module has no gpu dialect ops
# (the join runs inside libhj.so), so the gpu passes are no-ops and the CUDA
# runtime library is not needed; libhj.so brings its own HIP runtime.
set -euo pipefail
HERE=$(dirname "$(realpath -s "$0")")
ROOT=$(dirname "$HERE")
: "${LLVM_BUILD_DIR:=$HOME/llvm-project/build}"
: "${REF:=/root/reference}"
MLIR_OPT=$LLVM_BUILD_DIR/bin/mlir-opt
MLIR_CPU_RUNNER=$LLVM_BUILD_DIR/bin/mlir-cpu-runner
RUNNER_UTILS=$LLVM_BUILD_DIR/lib/libmlir_runner_utils.so
HJ=$ROOT/mlir-hashjoin_amd/lib/libhj.so
SHARED=${SHARED_SO:-$ROOT/oracle/_ref/shared.so}    # the reference's shared_stuff/shared.cpp
for f in "$MLIR_OPT" "$MLIR_CPU_RUNNER" "$RUNNER_UTILS" "$HJ" "$SHARED"; do
  [ -e "$f" ] || { echo "run_hj.sh: missing $f" >&2; exit 2; }
done
"$MLIR_OPT" -convert-scf-to-cf "$1" \
  | "$MLIR_OPT" -arith-expand \
  | "$MLIR_OPT" -convert-arith-to-llvm \
  | "$MLIR_OPT" -convert-cf-to-llvm \
  | "$MLIR_OPT" -finalize-memref-to-llvm \
  | "$MLIR_OPT" -convert-func-to-llvm \
  | "$MLIR_OPT" -reconcile-unrealized-casts \
  | "$MLIR_CPU_RUNNER" --shared-libs="$RUNNER_UTILS" --shared-libs="$HJ" --shared-libs="$SHARED" \
      --entry-point-result=void -O0
