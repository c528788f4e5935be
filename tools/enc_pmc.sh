#!/bin/bash
# PMC passes (separate, kernel-trace only) for the frame-level encoder kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/encpmc
export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  echo "== pass $i: $ctr"
  timeout -k 10 200 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/encpmc/p$i -o run -- python3 tools/bench_configs.py --configs enc --reps 3 > gpurun_out/encpmc/p$i.log 2>&1 || exit 1
done
echo "== done"
