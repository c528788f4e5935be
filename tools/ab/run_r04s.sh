# config 3 closed loop: DPP min / sum reductions (product) vs 9b085b8 (ds_bpermute)
set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests -m gpu > gpurun_out/pytest_gpu_r04s.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r04s.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r04s.log
LIBS="tools/_ab/libnanohevc_9b085b8.so nano-hevc_amd/nano_hevc/libnanohevc.so" CFG=closed TAG=r04s REPS=3 timeout -k 10 400 bash tools/ab/ab_libs.sh > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import json
lib=None
for l in open('gpurun_out/ab_libs_closed_r04s.jsonl'):
    d=json.loads(l)
    if 'rep' in d: lib=d['lib'].split('/')[-1]; continue
    print(lib, d.get('ms_per_frame'), d.get('roofline',{}).get('frac'))
PY
