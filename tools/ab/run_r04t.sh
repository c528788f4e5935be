# per-block calls and the config-5 int8 fix-up with DPP reductions: GPU tests, then the per-call cost
# of the product vs 6528b9c's build (tools/_ab/libnanohevc_9b085b8.so has the same block bodies), alternating
set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests -m gpu > gpurun_out/pytest_gpu_r04t.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r04t.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r04t.log
for rep in 1 2; do
  timeout -k 10 200 python tools/percall.py --lib tools/_ab/libnanohevc_9b085b8.so > gpurun_out/percall_old_r04t_$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python tools/percall.py > gpurun_out/percall_new_r04t_$rep.json 2>/dev/null || exit 1
done
tail -c 1500 gpurun_out/percall_new_r04t_2.json
