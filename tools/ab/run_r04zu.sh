# closed-loop config 4: the CTU-end recon gate at 2048 CTU rows vs the product's 4096, at 32 and 64 frames
set -o pipefail
R="--lib:tools/_ab/libnanohevc_gate2048.so product"
RUNS="$R" ARGS="--frames 32 --reps 10" TAG=r04zu_f32 REPS=3 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zu_f32.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04zu_f32.log
