#!/bin/bash
# One parameterised A/B session on the GPU box (replaces round 4's per-session
# run_r04*.sh scripts; VERDICT / ADVICE r4).  Steps run in the order given,
# each under its own time limit, stopping at the first failure:
#
#   TAG=r05x LIB=tools/_ab/libnanohevc_base.so bash tools/ab/session.sh tests:closed split:2 split:64 libs:4b
#
#   tests[:EXPR]   pytest -m gpu [-k EXPR] over tests/ (one process)
#   split:F        tools/ab/ab_closed4_split.sh at F frames: $LIB vs the product, REPS rounds
#                  (closed-loop config 4, luma / chroma / concurrent split timing)
#   libs:CFG       tools/ab/ab_libs.sh for bench_configs config CFG (3, closed, 4b, closed4, 5b): $LIB vs product
#   stamps:F       per-CTU stamps of the closed loop (A/B build, tools/ab/closed4_stamps.py) at F frames
#   cusplit        luma / chroma wavefronts on disjoint CU sets (ab_closed4_split.py --cu-split 0..3)
#   ktrace[:LIB]   kernel trace of the concurrent YUV420 call (tools/ab/closed4_trace.py): when each
#                  wavefront starts / ends inside the launch set (the product, or LIB copied over it)
# Outputs: gpurun_out/*_${TAG}*.  REPS (default 2), SPLIT_REPS (reps per run, default 10 at >= 16 frames, else 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:?set TAG}
REPS=${REPS:-2}
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"

step() {
  local name=${1%%:*} arg=
  [[ "$1" == *:* ]] && arg=${1#*:}
  case "$name" in
    tests)
      timeout -k 10 600 $PT tests -m gpu ${arg:+-k "$arg"} > gpurun_out/pytest_${TAG}.log 2>&1 \
        || { tail -30 gpurun_out/pytest_${TAG}.log; return 1; }
      tail -1 gpurun_out/pytest_${TAG}.log ;;
    split)
      local reps=${SPLIT_REPS:-$([ "$arg" -ge 16 ] && echo 10 || echo 5)}
      RUNS="--lib:${LIB:?set LIB} product" ARGS="--frames $arg --reps $reps" TAG=${TAG}_f$arg REPS=$REPS \
        timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_${TAG}_f$arg.log 2>&1 || return 1
      grep -v amdgpu.ids gpurun_out/ab_split_${TAG}_f$arg.log ;;
    libs)
      LIBS="${LIB:?set LIB} nano-hevc_amd/nano_hevc/libnanohevc.so" CFG=$arg TAG=$TAG REPS=$REPS \
        timeout -k 10 400 bash tools/ab/ab_libs.sh > gpurun_out/ab_libs_${TAG}_$arg.log 2>&1 || return 1
      tail -4 gpurun_out/ab_libs_${TAG}_$arg.log ;;
    stamps)
      NH_CLOSED4_STAMPS=1 timeout -k 10 200 python tools/ab/closed4_stamps.py --frames ${arg:-2} \
        > gpurun_out/stamps_${TAG}.json || return 1 ;;
    ktrace)
      local d=gpurun_out/kt_closed4_${TAG}${arg:+_$(basename $arg .so)}
      if [ -n "$arg" ]; then cp nano-hevc_amd/nano_hevc/libnanohevc.so /tmp/nh_product.so && cp "$arg" nano-hevc_amd/nano_hevc/libnanohevc.so; fi
      timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/ab/closed4_trace.py > $d.log 2>&1; local rc=$?
      if [ -n "$arg" ]; then cp /tmp/nh_product.so nano-hevc_amd/nano_hevc/libnanohevc.so; fi
      [ $rc -eq 0 ] || return 1
      python3 tools/ab/closed4_trace.py --summary $d ;;
    cusplit)
      local out=gpurun_out/ab_closed4_cusplit_${TAG}.jsonl
      for rep in $(seq $REPS); do
        for k in 0 1 2 3; do
          local a=""; [ $k -gt 0 ] && a="--cu-split $k"
          timeout -k 10 150 python tools/ab/ab_closed4_split.py --frames 64 --reps 10 $a >> $out || return 1
        done
      done ;;
    *)
      echo "unknown step $1"; return 2 ;;
  esac
}

for s in "$@"; do
  echo "== $s"
  step "$s" || { echo "== step $s failed; stopping"; exit 1; }
done
echo "== done"
