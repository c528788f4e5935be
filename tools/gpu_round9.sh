#!/bin/bash
# GPU session: closed-loop config 3 -- parity at both register allocations, then
# the closed leg at each (NH_CLOSED_WAVES 1 / 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01af}
echo "== pytest closed (1 wave)" && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "closed" > gpurun_out/pytest_closed_${TAG}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_closed_${TAG}.log; [ $rc -eq 0 ] && \
echo "== pytest closed (2 waves)" && \
NH_CLOSED_WAVES=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "closed" > gpurun_out/pytest_closed2_${TAG}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_closed2_${TAG}.log; [ $rc -eq 0 ] && \
echo "== closed (1 wave)" && \
timeout -k 10 300 python tools/bench_configs.py --configs closed > gpurun_out/closed1_${TAG}.jsonl 2> gpurun_out/closed1_${TAG}.err && cut -c1-260 gpurun_out/closed1_${TAG}.jsonl && \
echo "== closed (2 waves)" && \
NH_CLOSED_WAVES=2 timeout -k 10 300 python tools/bench_configs.py --configs closed > gpurun_out/closed2_${TAG}.jsonl 2> gpurun_out/closed2_${TAG}.err && cut -c1-260 gpurun_out/closed2_${TAG}.jsonl && \
echo "== done"
