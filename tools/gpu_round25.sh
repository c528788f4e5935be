#!/bin/bash
# Config 4 closed loop, batched dataflow rounds: parity (both register forms) + timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01bl}
for wv in 1 3; do
NH_TU_CLOSED_WAVES=$wv timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tu_pipeline_closed or closed_loop" > gpurun_out/pytest_c4b_${wv}_${TAG}.log 2>&1; rc=$?; echo "waves=$wv tests: $(tail -1 gpurun_out/pytest_c4b_${wv}_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_c4b_${wv}_${TAG}.log; exit 1; }
done
for wv in 1 3 1 3; do
  NH_TU_CLOSED_WAVES=$wv timeout -k 10 300 python tools/bench_configs.py --configs closed4 > gpurun_out/c4b_${wv}_${TAG}.jsonl 2> gpurun_out/c4b_${wv}_${TAG}.err || exit 1
  echo "waves=$wv $(python3 -c "import json; d=json.loads(open('gpurun_out/c4b_${wv}_${TAG}.jsonl').readline()); print(round(d['ms_per_frame'],4))")"
done
echo "== done"
