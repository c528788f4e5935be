#!/bin/bash
# XCD-aware workgroup order A/B for the hot kernel (variants 4096 + 16c + 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01aj}
echo "== pytest variants" && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "variants" > gpurun_out/pytest_var_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_var_${TAG}.log; [ $rc -eq 0 ] && \
echo "== A/B" && \
timeout -k 10 400 python tools/ab_fwd8x8.py --variants ${VARIANTS:-0,5,1,4101,4133,4165,4197,4341} --rounds 10 > gpurun_out/ab_xcd_${TAG}.json 2> gpurun_out/ab_xcd_${TAG}.err && python -c "
import json; d=json.load(open('gpurun_out/ab_xcd_${TAG}.json'))
for k,v in d['results'].items(): print(k, round(v['GBps_median']), round(v['GBps_best']), v.get('equal_v0',''))" && \
echo "== done"
