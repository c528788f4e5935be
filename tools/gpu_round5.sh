#!/bin/bash
# GPU session (re-entry check): smoke, full GPU parity suite, default bench,
# kernel-trace stats of the bench, config-3/4/5 legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01ae}
echo "== smoke" && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1; rc=$?; tail -2 gpurun_out/smoke_${TAG}.log; [ $rc -eq 0 ] && \
echo "== pytest -m gpu" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] && \
echo "== bench" && \
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err && cut -c1-2000 gpurun_out/bench_${TAG}.json && \
echo "== rocprof kernel-trace stats" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 && \
echo "== configs" && \
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err && cat gpurun_out/configs_${TAG}.jsonl && \
echo "== done"
