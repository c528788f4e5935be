#!/bin/bash
# PMC pass (SQ block) over the config-3 kernel: instruction mix and wave states.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01t}
echo "== pmc SQ" && \
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_cfg3_${TAG} -o run -- python3 tools/bench_configs.py --configs 3 --reps 2 > gpurun_out/pmc_cfg3_${TAG}.log 2>&1 && \
echo "== done"
