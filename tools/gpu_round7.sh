#!/bin/bash
# GPU session: config-3 chain rework -- parity at both register allocations,
# then the config-3 leg at each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01s}
echo "== pytest rdo (3 waves)" && \
NH_RDO_WAVES=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rdo" > gpurun_out/pytest_rdo3_${TAG}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_rdo3_${TAG}.log; [ $rc -eq 0 ] && \
echo "== configs 3 (default)" && \
timeout -k 10 300 python tools/bench_configs.py --configs 3 > gpurun_out/configs3_${TAG}.jsonl 2> gpurun_out/configs3_${TAG}.err && cut -c1-200 gpurun_out/configs3_${TAG}.jsonl && \
echo "== configs 3 (3 waves)" && \
NH_RDO_WAVES=3 timeout -k 10 300 python tools/bench_configs.py --configs 3 > gpurun_out/configs3w_${TAG}.jsonl 2> gpurun_out/configs3w_${TAG}.err && cut -c1-200 gpurun_out/configs3w_${TAG}.jsonl && \
echo "== done"
