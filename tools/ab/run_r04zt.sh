# closed-loop config 4: whole-CTU level rows too (int16 in LDS, 16-B pieces at the CTU end) vs 6367547
set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests -m gpu -k "closed or tu_pipeline" > gpurun_out/pytest_closed_r04zt.log 2>&1 || { tail -30 gpurun_out/pytest_closed_r04zt.log; exit 1; }
tail -1 gpurun_out/pytest_closed_r04zt.log
R="--lib:tools/_ab/libnanohevc_6367547.so product"
RUNS="$R" ARGS="--frames 2 --reps 5" TAG=r04zt_f2 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zt_f2.log 2>&1 || exit 1
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04zt_f64 REPS=3 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zt_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04zt_f2.log gpurun_out/ab_split_r04zt_f64.log
