# closed-loop config 4: the rounds loop walks only the non-empty (round, size) entries (product) vs cc0ca14
set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests -m gpu -k "closed" > gpurun_out/pytest_closed_r04zd.log 2>&1 || { tail -30 gpurun_out/pytest_closed_r04zd.log; exit 1; }
tail -1 gpurun_out/pytest_closed_r04zd.log
R="--lib:tools/_ab/libnanohevc_cc0ca14.so product"
RUNS="$R" ARGS="--frames 2 --reps 5" TAG=r04zd_f2 REPS=3 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zd_f2.log 2>&1 || exit 1
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04zd_f64 REPS=3 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zd_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04zd_f2.log gpurun_out/ab_split_r04zd_f64.log
