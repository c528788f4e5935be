set -o pipefail
TAG=r04j bash tools/gpu_run.sh tests || exit 1
RUNS="--lib:tools/_ab/libnanohevc_head.so product" ARGS="--frames 2 --reps 5" TAG=r04j_f2 REPS=2 timeout -k 10 400 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04j_f2.log 2>&1 || exit 1
RUNS="--lib:tools/_ab/libnanohevc_head.so product" ARGS="--frames 64 --reps 10" TAG=r04j_f64 REPS=2 timeout -k 10 400 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04j_f64.log 2>&1 || exit 1
LIBS="tools/_ab/libnanohevc_head.so nano-hevc_amd/nano_hevc/libnanohevc.so" CFG=4b TAG=r04j REPS=2 timeout -k 10 300 bash tools/ab/ab_libs.sh > /dev/null 2>&1 || exit 1
LIBS="tools/_ab/libnanohevc_head.so nano-hevc_amd/nano_hevc/libnanohevc.so" CFG=5b TAG=r04j REPS=2 timeout -k 10 300 bash tools/ab/ab_libs.sh > /dev/null 2>&1 || exit 1
NH_CLOSED4_STAMPS=1 timeout -k 10 200 python tools/ab/closed4_stamps.py --frames 2 > gpurun_out/stamps_r04j.json || exit 1
tail -6 gpurun_out/ab_split_r04j_f2.log gpurun_out/ab_split_r04j_f64.log
