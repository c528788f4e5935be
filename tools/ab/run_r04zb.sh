# closed-loop config 4, like-for-like product builds (the r04q / r04o "--ab" runs compared the A/B library,
# itself ~25 % slower through its probe and stamp paths, with the product):
#   srcdma0/1/2: 5fa8d8e with NH_CLOSED4_SRC_DMA defaulting to 0 / 1 (luma + chroma) / 2 (luma)
#   mfma32off:   HEAD with the 32x32 luma TUs on the packed chain instead of the f16 matrix cores
set -o pipefail
R="--lib:tools/_ab/libnanohevc_srcdma0.so --lib:tools/_ab/libnanohevc_srcdma1.so --lib:tools/_ab/libnanohevc_srcdma2.so --lib:tools/_ab/libnanohevc_mfma32off.so product"
RUNS="$R" ARGS="--frames 2 --reps 5" TAG=r04zb_f2 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zb_f2.log 2>&1 || exit 1
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04zb_f64 REPS=2 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zb_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04zb_f2.log gpurun_out/ab_split_r04zb_f64.log
