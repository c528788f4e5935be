# Instruction-cache pass (SQC_ICACHE_* + SQ_IFETCH + SQ_WAIT_INST_ANY) of bench_configs configs on the
# product library:  TAG=x CFGS="closed4 3" bash tools/ab/pmc_icache.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in $CFGS; do
  echo "== $c" >> gpurun_out/pmc_icache_${TAG}.log
  timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES --output-format csv -d gpurun_out/pmc_icache_${TAG}_$c -o run -- python3 tools/bench_configs.py --configs $c --reps 3 $ARGS >> gpurun_out/pmc_icache_${TAG}.log 2>&1 || exit 1
done
