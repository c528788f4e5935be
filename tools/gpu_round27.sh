#!/bin/bash
# Config 4 closed loop: luma/chroma wavefronts concurrent on two streams -- parity + batch sweep (sequential vs concurrent).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01br}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "closed" > gpurun_out/pytest_c4conc_${TAG}.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pytest_c4conc_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_c4conc_${TAG}.log; exit 1; }
for nf in 16 32 64; do for m in seq conc; do
  fl=""; [ $m = seq ] && fl="--closed4-seq"
  timeout -k 10 150 python tools/bench_configs.py --configs closed4 --closed4-frames $nf --reps 8 $fl > gpurun_out/c4_${m}_${nf}_${TAG}.jsonl 2> gpurun_out/c4_${m}_${nf}_${TAG}.err || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/c4_${m}_${nf}_${TAG}.jsonl').read().splitlines()[-1]); print('$m', $nf, round(d['ms_per_launch_set'],3), round(d['ms_per_frame'],4))"
done; done
echo "== done"
