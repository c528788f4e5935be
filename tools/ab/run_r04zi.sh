# closed-loop config 4 at 64 frames, A/B library against itself: timing probes 0 (full), 64 (no level /
# recon / TU-map stores in the chains), 32 (no source loads) -- upper bounds for store / load work
set -o pipefail
R="--ab:NH_CLOSED4_PROBE=0 --ab:NH_CLOSED4_PROBE=64 --ab:NH_CLOSED4_PROBE=32"
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04zi_f64 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zi_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04zi_f64.log
