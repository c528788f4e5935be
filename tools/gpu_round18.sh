#!/bin/bash
# Closed loop: ticket order A/B (NH_CLOSED_ORDER 1 row-major across planes, 0 plane-major) + parity in both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01ay}
for o in 1 0; do
  NH_CLOSED_ORDER=$o timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "closed" > gpurun_out/pytest_closed_o${o}_${TAG}.log 2>&1; rc=$?; echo "order=$o $(tail -1 gpurun_out/pytest_closed_o${o}_${TAG}.log)"; [ $rc -eq 0 ] || exit 1
done
for o in 1 0 1 0; do
  NH_CLOSED_ORDER=$o timeout -k 10 300 python tools/bench_configs.py --configs closed > gpurun_out/closed_o${o}_${TAG}.jsonl 2> gpurun_out/closed_o${o}_${TAG}.err || exit 1
  echo "order=$o $(cut -c150-330 gpurun_out/closed_o${o}_${TAG}.jsonl)"
done
echo "== done"
