# closed-loop config 4: CTU source staged in LDS by LDS-DMA (A/B knob NH_CLOSED4_SRC_DMA: 1 luma + chroma,
# 2 luma only) vs the product (unstaged); parity of the staged forms on the A/B library first
set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
NH_TEST_AB=1 NH_CLOSED4_SRC_DMA=1 timeout -k 10 300 $PT tests -m gpu -k "closed" > gpurun_out/pytest_srcdma_r04q.log 2>&1 || { tail -30 gpurun_out/pytest_srcdma_r04q.log; exit 1; }
tail -2 gpurun_out/pytest_srcdma_r04q.log
R="product --ab:NH_CLOSED4_SRC_DMA=1 --ab:NH_CLOSED4_SRC_DMA=2"
RUNS="$R" ARGS="--frames 2 --reps 5" TAG=r04q_f2 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04q_f2.log 2>&1 || exit 1
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04q_f64 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04q_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04q_f2.log gpurun_out/ab_split_r04q_f64.log
