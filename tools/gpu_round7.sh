#!/bin/bash
# GPU session: config-3/4/5 kernels -- parity (small + full size), then the
# config legs; config 3 at each launch form (NH_RDO_FORM 0/1/2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01ag}
echo "== pytest rdo/tu/tc32 + full size" && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rdo or closed or cfg or tu_ or tc32" > gpurun_out/pytest_rdo_${TAG}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_rdo_${TAG}.log; [ $rc -eq 0 ] && \
echo "== configs 3,closed,4b" && \
timeout -k 10 300 python tools/bench_configs.py --configs 4b,4 > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err && cut -c1-220 gpurun_out/configs_${TAG}.jsonl && \
echo "== done"
