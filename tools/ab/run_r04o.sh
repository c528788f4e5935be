# closed-loop config 4: 7eaa0ee / per-lane offset only (pyx) / offset + no `on` guards /
# product (offset + guards + chroma without LDS bases) / A/B lib with luma bases from global too
set -o pipefail
TAG=r04o bash tools/gpu_run.sh tests || exit 1
R="--lib:tools/_ab/libnanohevc_7eaa0ee.so --lib:tools/_ab/libnanohevc_pyx.so --lib:tools/_ab/libnanohevc_noguard.so product --ab:NH_CLOSED4_BASIS_GLOBAL=1"
RUNS="$R" ARGS="--frames 2 --reps 5" TAG=r04o_f2 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04o_f2.log 2>&1 || exit 1
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04o_f64 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04o_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04o_f2.log gpurun_out/ab_split_r04o_f64.log
