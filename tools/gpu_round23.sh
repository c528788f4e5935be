#!/bin/bash
# Closed loops with wave-level LDS sync instead of __syncthreads: parity + timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01bj}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "closed" > gpurun_out/pytest_wsync_${TAG}.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pytest_wsync_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_wsync_${TAG}.log; exit 1; }
for r in 1 2; do
timeout -k 10 300 python tools/bench_configs.py --configs closed,closed4 > gpurun_out/wsync_${TAG}_$r.jsonl 2> gpurun_out/wsync_${TAG}_$r.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/wsync_${TAG}_$r.jsonl'):
    d=json.loads(l); print(d['config'][:24], round(d['ms_per_frame'],4))"
done
echo "== done"
