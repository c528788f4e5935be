# closed-loop config 4: luma waves at s_setprio 3 (A/B probe bit 128) vs 2 (product)
set -o pipefail
R="product --ab:NH_CLOSED4_PROBE=128"
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04za_f64 REPS=3 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04za_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04za_f64.log
