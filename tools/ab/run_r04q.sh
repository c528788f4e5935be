# closed-loop config 4: CTU source staged in LDS by LDS-DMA, luma + chroma (product) / luma only / off (A/B knob) / 7eaa0ee
set -o pipefail
TAG=r04q bash tools/gpu_run.sh tests || exit 1
R="--lib:tools/_ab/libnanohevc_7eaa0ee.so product --ab:NH_CLOSED4_SRC_DMA=2 --ab:NH_CLOSED4_SRC_DMA=0"
RUNS="$R" ARGS="--frames 2 --reps 5" TAG=r04q_f2 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04q_f2.log 2>&1 || exit 1
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04q_f64 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04q_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04q_f2.log gpurun_out/ab_split_r04q_f64.log
