#!/bin/bash
# PMC pass (SQ block) over the config-3 kernel: instruction mix and wave states.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01ad}
echo "== pmc SQ" && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_cfg3_${TAG} -o run -- python3 tools/bench_configs.py --configs 3 --reps 2 > gpurun_out/pmc_cfg3_${TAG}.log 2>&1 && \
echo "== done"
