#!/bin/bash
# Closed loop: tagged-line form (default) parity + A/B against the progress-counter form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01ax}
echo "== pytest closed (tagged)" && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "closed" > gpurun_out/pytest_closed_${TAG}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_closed_${TAG}.log; [ $rc -eq 0 ] || exit 1
for f in 1 0 1 0; do
  NH_CLOSED_FORM=$f timeout -k 10 300 python tools/bench_configs.py --configs closed > gpurun_out/closed_f${f}_${TAG}.jsonl 2> gpurun_out/closed_f${f}_${TAG}.err || exit 1
  echo "form=$f $(cut -c1-300 gpurun_out/closed_f${f}_${TAG}.jsonl)"
done
echo "== done"
