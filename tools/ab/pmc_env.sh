# One SQ counter pass (tools/gpu_run.sh valu_pmc1's counters) of a bench_configs config on the A/B
# library per environment setting:  TAG=x CFG=3 ENVS="NH_X=0|NH_X=1" bash tools/ab/pmc_env.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS='|' read -r -a SETS <<< "$ENVS"
i=0
for e in "${SETS[@]}"; do
  i=$((i + 1))
  echo "== $e" >> gpurun_out/pmc_env_${TAG}.log
  env $e timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_env_${TAG}_$i -o run -- python3 tools/bench_configs.py --ab --configs $CFG --reps 3 >> gpurun_out/pmc_env_${TAG}.log 2>&1 || exit 1
done
