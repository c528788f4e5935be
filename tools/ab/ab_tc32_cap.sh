set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for rep in 1 2; do for c in 3 4; do
  echo "{\"cap_c\": $c, \"rep\": $rep}" >> gpurun_out/ab_cap_r06c.jsonl
  NH_TC32H_CAP_C=$c timeout -k 10 200 python tools/bench_configs.py --ab --configs 5b --cfg5-levels int16,int8 --reps 20 >> gpurun_out/ab_cap_r06c.jsonl 2>> gpurun_out/ab_cap_r06c.err || exit 1
done; done
