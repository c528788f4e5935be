#!/bin/bash
# Closed loop: lane-pair form (NH_CLOSED_FORM=2) parity + A/B against the tagged form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01ba}
NH_CLOSED_FORM=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "closed" > gpurun_out/pytest_closed_pair_${TAG}.log 2>&1; rc=$?; echo "pair: $(tail -1 gpurun_out/pytest_closed_pair_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_closed_pair_${TAG}.log; exit 1; }
for fw in "1 1" "2 2" "2 3" "1 1" "2 2" "2 3"; do
  set -- $fw
  NH_CLOSED_FORM=$1 NH_CLOSED_WAVES=$2 timeout -k 10 300 python tools/bench_configs.py --configs closed > gpurun_out/closed_pf$1w$2_${TAG}.jsonl 2> gpurun_out/closed_pf$1w$2_${TAG}.err || exit 1
  echo "form=$1 waves=$2 $(cut -c150-260 gpurun_out/closed_pf$1w$2_${TAG}.jsonl)"
done
echo "== done"
