# closed-loop config 4: pk2 without `on` guards and with one per-lane offset (product) vs 7eaa0ee
set -o pipefail
TAG=r04n bash tools/gpu_run.sh tests || exit 1
RUNS="--lib:tools/_ab/libnanohevc_7eaa0ee.so product" ARGS="--frames 2 --reps 5" TAG=r04n_f2 REPS=2 timeout -k 10 400 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04n_f2.log 2>&1 || exit 1
RUNS="--lib:tools/_ab/libnanohevc_7eaa0ee.so product" ARGS="--frames 64 --reps 10" TAG=r04n_f64 REPS=2 timeout -k 10 400 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04n_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04n_f2.log gpurun_out/ab_split_r04n_f64.log
