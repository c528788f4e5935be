#!/bin/bash
# PMC pass (SQ block) over the config-4 closed loop (k_tu_closed, dataflow rounds): wave states, instruction mix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01bq}
echo "== pmc SQ closed4 (pass 1)" && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_closed4_${TAG} -o run -- python3 tools/bench_configs.py --configs closed4 --reps 2 > gpurun_out/pmc_closed4_${TAG}.log 2>&1 && \
echo "== pmc SQ closed4 (pass 2)" && \
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmc2_closed4_${TAG} -o run -- python3 tools/bench_configs.py --configs closed4 --reps 2 > gpurun_out/pmc2_closed4_${TAG}.log 2>&1 ; \
echo "== done"
