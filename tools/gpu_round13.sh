#!/bin/bash
# XCD-aware order: hot kernel + linear copy A/B, frame driver / casts with NH_XCD_ORDER=0/1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01an}
echo "== frame parity" && \
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "frame or encode or widen or narrow or variants" > gpurun_out/pytest_xcd_${TAG}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_xcd_${TAG}.log; [ $rc -eq 0 ] || exit 1
echo "== A/B" && \
timeout -k 10 400 python tools/ab_fwd8x8.py --variants 0,5,4341 --xcd --epilogue --rounds 10 > gpurun_out/ab_xcd_${TAG}.json 2> gpurun_out/ab_xcd_${TAG}.err && python -c "
import json; d=json.load(open('gpurun_out/ab_xcd_${TAG}.json'))
for k,v in d['results'].items(): print(k, round(v['GBps_median']), round(v['GBps_best']), v.get('equal_v0',''))" || exit 1
for r in 1 2; do for x in 0 1; do
  NH_XCD_ORDER=$x timeout -k 10 200 python tools/bench_configs.py --configs enc,io > gpurun_out/cfg_xcd${x}_${TAG}_$r.jsonl 2> gpurun_out/cfg_xcd${x}_${TAG}_$r.err || exit 1
  python -c "
import json
for l in open('gpurun_out/cfg_xcd${x}_${TAG}_$r.jsonl'):
    d=json.loads(l); print('xcd=$x', d.get('config','')[:20], d.get('ms_per_launch'), d.get('roofline',{}).get('frac'), d.get('frac_widen'), d.get('frac_narrow'))"
done; done
echo "== done"
