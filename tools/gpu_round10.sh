#!/bin/bash
# Full-size reference parity (tests/test_fullsize_reference_gpu.py) + the store-policy A/B variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01ai}
echo "== pytest fullsize reference" && \
timeout -k 10 600 python -u -m pytest tests/test_fullsize_reference_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_fullref_${TAG}.log 2>&1; rc=$?; tail -12 gpurun_out/pytest_fullref_${TAG}.log; [ $rc -eq 0 ] && \
echo "== done"
