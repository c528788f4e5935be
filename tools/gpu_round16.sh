#!/bin/bash
# PMC passes on tools/tlb_probe.py: translation misses for the slow vs fast output placement.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01aw}
timeout -k 10 120 python tools/tlb_probe.py > gpurun_out/tlb_plain_${TAG}.json 2>&1 && cat gpurun_out/tlb_plain_${TAG}.json || exit 1
rocprofv3 --list-avail > gpurun_out/pmc_avail_${TAG}.txt 2>&1 || true
grep -io "[A-Z_0-9]*UTCL[A-Z_0-9]*\|[A-Z_0-9]*TLB[A-Z_0-9]*\|[A-Z_0-9]*TRANSLATION[A-Z_0-9]*" gpurun_out/pmc_avail_${TAG}.txt | sort -u | head -40 || true
for c in ${COUNTERS:-TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum}; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_tlb_${TAG}_$c -o run -- python3 tools/tlb_probe.py > gpurun_out/pmc_tlb_${TAG}_$c.log 2>&1 || { echo "pass $c failed"; tail -5 gpurun_out/pmc_tlb_${TAG}_$c.log; exit 1; }
  python3 -c "
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/pmc_tlb_${TAG}_$c/run_counter_collection.csv')) if 'k_fwd8x8' in r['Kernel_Name']]
print('$c', [round(float(r['Counter_Value'])) for r in rows])"
done
echo "== done"
