#!/bin/bash
# Config 4: TU-size launches forked onto side streams -- parity + A/B (NH_TU_STREAMS=0/1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01bc}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tu_ or cfg4 or tu32" > gpurun_out/pytest_tu_${TAG}.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pytest_tu_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_tu_${TAG}.log; exit 1; }
for t in 1 0 1 0; do
  NH_TU_STREAMS=$t timeout -k 10 300 python tools/bench_configs.py --configs 4,4b > gpurun_out/cfg4_s${t}_${TAG}.jsonl 2> gpurun_out/cfg4_s${t}_${TAG}.err || exit 1
  python3 -c "
import json
for l in open('gpurun_out/cfg4_s${t}_${TAG}.jsonl'):
    d=json.loads(l); print('streams=$t', d['config'][:14], round(d['ms_per_frame'],4))"
done
echo "== done"
