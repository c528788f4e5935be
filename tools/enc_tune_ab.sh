#!/bin/bash
# Parity of the pipelined encoder form (small cap => many passes per workgroup)
# and a sweep of NH_ENC_TUNE launch shapes on the 64-frame 4K bench leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NH_ENC_TUNE=2,1,1,64 timeout -k 10 300 python -m pytest tests/test_frame_gpu.py -m gpu -x -q > gpurun_out/pf_pipe.log 2>&1; rc=$?; tail -2 gpurun_out/pf_pipe.log; [ $rc -eq 0 ] || exit 1
for t in ${TUNES:-4,2,0,0 4,2,1,2048 2,1,1,2048 1,1,1,2048 2,1,1,4096 4,1,1,1024 2,2,1,2048 4,1,1,4096}; do
  NH_ENC_TUNE=$t timeout -k 10 120 python tools/bench_configs.py --configs enc 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', round(d['ms_per_launch'],3), round(d['roofline']['frac'],3))" || exit 1
done
