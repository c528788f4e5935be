#!/bin/bash
# Config 4 32x32 TUs: compacted tree walk in k_tc32_mfma -- parity + timing (NH_TC32_TREE_WAVES 1 / 4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01bo}
for wv in 1 4; do
NH_TC32_TREE_WAVES=$wv timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py tests/test_fullsize_reference_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tu_ or cfg4 or tc32 or cfg5" > gpurun_out/pytest_tc32t_${wv}_${TAG}.log 2>&1; rc=$?; echo "waves=$wv tests: $(tail -1 gpurun_out/pytest_tc32t_${wv}_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_tc32t_${wv}_${TAG}.log; exit 1; }
done
for wv in 1 4 1 4; do
  NH_TC32_TREE_WAVES=$wv timeout -k 10 300 python tools/bench_configs.py --configs 4b,5 > gpurun_out/tc32t_${wv}_${TAG}.jsonl 2> gpurun_out/tc32t_${wv}_${TAG}.err || exit 1
  python3 -c "
import json
for l in open('gpurun_out/tc32t_${wv}_${TAG}.jsonl'):
    d=json.loads(l); print('waves=$wv', d['config'][:22], d.get('ms_per_frame', (d.get('mfma_i8') or {}).get('ms_per_frame')))"
done
echo "== done"
