#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel-trace stats and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE separately, per MI355X_MICROARCH.md §HBM).
# Every GPU step has its own time limit; steps are chained with && so the
# script stops at the first failure.  Outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
STEPS=${STEPS:-20}
FRAMES=${FRAMES:-128}
echo "== pytest -m gpu" && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] && \
echo "== bench" && \
timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 --frames $FRAMES > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err && cat gpurun_out/bench_${TAG}.json && \
echo "== rocprof kernel-trace stats" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps $STEPS --warmup 5 --frames $FRAMES --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 && \
echo "== rocprof pmc FETCH_SIZE" && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o run -- python3 bench.py --steps 5 --warmup 2 --frames $FRAMES --no-cpu-baseline > gpurun_out/pmc_fetch_${TAG}.log 2>&1 && \
echo "== rocprof pmc WRITE_SIZE" && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${TAG} -o run -- python3 bench.py --steps 5 --warmup 2 --frames $FRAMES --no-cpu-baseline > gpurun_out/pmc_write_${TAG}.log 2>&1 && \
echo "== done" && find gpurun_out -name "*.csv" | head -50
