#!/bin/bash
# GPU session: full-size parity (configs 2-5 at BASELINE sizes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01v}
echo "== pytest full size" && \
timeout -k 10 600 python -u -m pytest tests/test_full_size_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_full_${TAG}.log 2>&1; rc=$?; tail -12 gpurun_out/pytest_full_${TAG}.log; [ $rc -eq 0 ] && \
echo "== done"
