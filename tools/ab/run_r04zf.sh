# closed-loop config 4: one copy of the 32x32 MFMA chain's code (a plane loop) vs 60717be (two inlined copies)
set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests -m gpu -k "closed" > gpurun_out/pytest_closed_r04zf.log 2>&1 || { tail -30 gpurun_out/pytest_closed_r04zf.log; exit 1; }
tail -1 gpurun_out/pytest_closed_r04zf.log
R="--lib:tools/_ab/libnanohevc_60717be.so product"
RUNS="$R" ARGS="--frames 2 --reps 5" TAG=r04zf_f2 REPS=3 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zf_f2.log 2>&1 || exit 1
RUNS="$R" ARGS="--frames 64 --reps 10" TAG=r04zf_f64 REPS=3 timeout -k 10 500 bash tools/ab/ab_closed4_split.sh > gpurun_out/ab_split_r04zf_f64.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_split_r04zf_f2.log gpurun_out/ab_split_r04zf_f64.log
# instruction-cache behaviour of the two builds (closed4 at 64 frames; one counter pass each)
for lib in tools/_ab/libnanohevc_60717be.so nano-hevc_amd/nano_hevc/libnanohevc.so; do
  tag=$(basename $lib .so)
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES --output-format csv -d gpurun_out/icache_r04zf_$tag -o run -- python3 tools/bench_configs.py --configs closed4 --reps 3 --lib $lib > gpurun_out/icache_r04zf_$tag.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/icache_r04zf_*/")):
    tot = collections.Counter()
    for p in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "closed_pair" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    h, m = tot["SQC_ICACHE_HITS"], tot["SQC_ICACHE_MISSES"]
    print(d, dict(tot), "miss rate", m / max(1.0, h + m))
PY
