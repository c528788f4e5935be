#!/bin/bash
# A/B of whole library builds over a bench_configs config, alternating processes:
#   LIBS="nano-hevc_amd/nano_hevc/libnanohevc.so tools/_ab/libnanohevc_pre_srcimg.so" CFG=closed4 TAG=x tools/ab/ab_libs.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${TAG:-ab}
REPS=${REPS:-3}
ARGS=${ARGS:-"--reps 8"}
OUT=gpurun_out/ab_libs_${CFG}_${TAG}.jsonl
for rep in $(seq $REPS); do
  for lib in $LIBS; do
    echo "{\"lib\": \"$lib\", \"rep\": $rep}" >> $OUT
    timeout -k 10 150 python tools/bench_configs.py --lib $lib --configs $CFG $ARGS >> $OUT || exit 1
  done
done
cat $OUT
