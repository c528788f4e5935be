#!/bin/bash
# GPU session: parity tests, default bench, 2-rank gloo rehearsal of the
# multi-rank bench path on the one GPU, rocprof stats + PMC passes (default variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01c}
echo "== pytest -m gpu" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] && \
echo "== bench" && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err && cat gpurun_out/bench_${TAG}.json && \
echo "== 2-rank rehearsal (gloo, shared GPU)" && \
NH_DIST_BACKEND=gloo NH_FORCE_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --frames 16 --gather-steps 1 > gpurun_out/bench2_${TAG}.json 2> gpurun_out/bench2_${TAG}.err && cat gpurun_out/bench2_${TAG}.json && \
echo "== rocprof kernel-trace stats" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1 && \
echo "== rocprof pmc FETCH_SIZE" && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_fetch_${TAG}.log 2>&1 && \
echo "== rocprof pmc WRITE_SIZE" && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${TAG} -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_write_${TAG}.log 2>&1 && \
echo "== done"
