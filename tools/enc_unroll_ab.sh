set -o pipefail
mkdir -p gpurun_out/encab
export TMPDIR=/tmp
for u in "4,2" "2,1" "4,1" "4,4" "2,2" "1,1"; do
  echo "== $u"
  NH_ENC_UNROLL=$u timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/encab/u${u/,/_} -o run -- python3 tools/bench_configs.py --configs enc --reps 5 > gpurun_out/encab/u${u/,/_}.log 2>&1 || exit 1
  grep -h encode gpurun_out/encab/u${u/,/_}/run_kernel_stats.csv | cut -d, -f1-4
done
