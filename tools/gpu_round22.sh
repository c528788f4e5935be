#!/bin/bash
# Config 4 closed loop: parity + bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01bh}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "closed" > gpurun_out/pytest_closed4_${TAG}.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pytest_closed4_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_closed4_${TAG}.log; exit 1; }
timeout -k 10 300 python tools/bench_configs.py --configs closed4 ${CHECK:-} > gpurun_out/closed4_${TAG}.jsonl 2> gpurun_out/closed4_${TAG}.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/closed4_${TAG}.jsonl'):
    d=json.loads(l); print(d['config'][:20], round(d['ms_per_frame'],4), d.get('frame0_luma_equals_oracle',''))"
echo "== done"
