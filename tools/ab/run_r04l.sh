# closed-loop config 4: the explicit pre-rounds vmcnt(0) (product) vs 3f433dd, and the per-phase batch stamps
set -o pipefail
RUNS="--lib:tools/_ab/libnanohevc_3f433dd.so product" ARGS="--frames 2 --reps 5" TAG=r04l_f2 REPS=2 timeout -k 10 400 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04l_f2.log 2>&1 || exit 1
RUNS="--lib:tools/_ab/libnanohevc_3f433dd.so product" ARGS="--frames 64 --reps 10" TAG=r04l_f64 REPS=2 timeout -k 10 400 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04l_f64.log 2>&1 || exit 1
NH_CLOSED4_MFMA32=0 NH_CLOSED4_STAMPS=1 timeout -k 10 200 python tools/ab/closed4_stamps.py --frames 2 > gpurun_out/stamps_r04l.json || exit 1
NH_CLOSED4_STAMPS=1 timeout -k 10 200 python tools/ab/closed4_stamps.py --frames 2 >> gpurun_out/stamps_r04l.json || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04l_f2.log gpurun_out/ab_split_r04l_f64.log
