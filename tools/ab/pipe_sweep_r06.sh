# Config-4 closed loop: launch sets pipelined over stream pairs (tools/ab/ab_closed4_split.py --pipe/--depth)
#   CASES="--frames 64 --pipe 6 --depth 3|..." TAG=x bash tools/ab/pipe_sweep_r06.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
O=gpurun_out/ab_closed4_pipe_${TAG}.jsonl
IFS='|' read -r -a CS <<< "$CASES"
for a in "${CS[@]}"; do
  timeout -k 10 200 python tools/ab/ab_closed4_split.py --reps 7 $a >> $O || exit 1
done
python3 - $O <<'PY'
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(d["frames"], *(f"{k} {d[k]['median_ms_per_frame']:.4f}" for k in d if isinstance(d[k],dict) and "median_ms_per_frame" in d[k]))
PY
