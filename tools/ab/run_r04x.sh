# closed-loop config 4 over YUV420: luma / chroma wavefronts on disjoint CU sets (gpu.CLOSED4_CU_SPLIT = k:
# chroma on CUs with index % 8 < k) vs both on every CU; alternating processes
set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests -m gpu -k "closed" > gpurun_out/pytest_cusplit_r04x.log 2>&1 || { tail -30 gpurun_out/pytest_cusplit_r04x.log; exit 1; }
tail -2 gpurun_out/pytest_cusplit_r04x.log
OUT=gpurun_out/ab_closed4_cusplit_r04x.jsonl
for rep in 1 2; do
  for k in 0 1 2 3; do
    A=""; [ $k -gt 0 ] && A="--cu-split $k"
    timeout -k 10 150 python tools/ab/ab_closed4_split.py --frames 64 --reps 10 $A >> $OUT || exit 1
  done
done
python3 - "$OUT" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d.get("cu_split"), *(f"{k} {d[k]['median_ms_per_frame']:.4f}" for k in ("luma", "chroma", "concurrent") if k in d), d["out_digest"])
PY
