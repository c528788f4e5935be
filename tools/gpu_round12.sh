#!/bin/bash
# bench.py per launch variant, alternating processes (XCD order A/B in the bench's own setting).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01am}
for r in 1 2; do
for v in ${VARIANTS:-5 4341 4229}; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --variant $v > gpurun_out/benchv_${TAG}_${v}_$r.json 2>gpurun_out/benchv_${TAG}_${v}_$r.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/benchv_${TAG}_${v}_$r.json')); print($v, $r, round(d['roofline']['achieved']), round(d['roofline']['frac'],4))"
done
done
echo "== done"
