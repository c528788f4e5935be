#!/bin/bash
# GPU session: config-3 kernels -- parity (small + full size), then the
# config-3 legs (open and closed loop) at both register allocations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01w}
echo "== pytest rdo" && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rdo or closed or cfg3" > gpurun_out/pytest_rdo_${TAG}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_rdo_${TAG}.log; [ $rc -eq 0 ] && \
echo "== configs 3 (default)" && \
timeout -k 10 300 python tools/bench_configs.py --configs 3,closed > gpurun_out/configs3_${TAG}.jsonl 2> gpurun_out/configs3_${TAG}.err && cut -c1-200 gpurun_out/configs3_${TAG}.jsonl && \
echo "== configs 3 (3 waves)" && \
NH_RDO_WAVES=3 timeout -k 10 300 python tools/bench_configs.py --configs 3 > gpurun_out/configs3w_${TAG}.jsonl 2> gpurun_out/configs3w_${TAG}.err && cut -c1-200 gpurun_out/configs3w_${TAG}.jsonl && \
echo "== done"
