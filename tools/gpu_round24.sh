#!/bin/bash
# Config 3 open loop: packed-only launch + fallback (NH_RDO_FORM=0) vs one launch (3): parity + timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01bk}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py tests/test_fullsize_reference_gpu.py tests/test_reference_scenarios_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rdo or cfg3" > gpurun_out/pytest_rdo2_${TAG}.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/pytest_rdo2_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_rdo2_${TAG}.log; exit 1; }
for f in 0 3 0 3; do
  NH_RDO_FORM=$f timeout -k 10 300 python tools/bench_configs.py --configs 3 > gpurun_out/rdo_f${f}_${TAG}.jsonl 2> gpurun_out/rdo_f${f}_${TAG}.err || exit 1
  echo "form=$f $(python3 -c "import json; d=json.loads(open('gpurun_out/rdo_f${f}_${TAG}.jsonl').readline()); print(round(d['ms_per_frame'],4))")"
done
echo "== done"
