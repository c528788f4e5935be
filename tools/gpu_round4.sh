#!/bin/bash
# GPU session: frame-level rows (encode_frame_intra driver, frame I/O casts) --
# parity tests, config bench legs, kernel stats; then the default bench (cpu
# baseline now with the all-threads leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01j}
echo "== pytest frame rows" && \
timeout -k 10 600 python -m pytest tests/test_frame_gpu.py -m gpu -x -q > gpurun_out/pytest_frame_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_frame_${TAG}.log; [ $rc -eq 0 ] && \
echo "== bench_configs enc,io" && \
timeout -k 10 300 python tools/bench_configs.py --configs enc,io > gpurun_out/configs_enc_${TAG}.jsonl 2> gpurun_out/configs_enc_${TAG}.err && cat gpurun_out/configs_enc_${TAG}.jsonl && \
echo "== rocprof enc,io" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enc_${TAG} -o run -- python3 tools/bench_configs.py --configs enc,io --reps 5 > gpurun_out/prof_enc_${TAG}.log 2>&1 && \
echo "== bench" && \
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err && cut -c1-1500 gpurun_out/bench_${TAG}.json && \
echo "== pytest -m gpu (all)" && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] && \
echo "== done"
