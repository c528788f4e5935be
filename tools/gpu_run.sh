#!/bin/bash
# The one GPU-session runner (replaces round 1's per-session gpu_roundN.sh).
#   TAG=r02a tools/gpu_run.sh STEP [STEP ...]
# Steps (run in the order given, each under its own time limit, stopping at the
# first failure; outputs under gpurun_out/):
#   tests      pytest -m gpu over tests/ (one process)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py (default line: N=1, cfg 2 hot path, cpu_baseline)
#   bench4     bench.py --config 4 (CTU-sharded config 4, N=1)
#   rehearse2  bench.py --gpus 2 on the one GPU (gloo, both ranks on device 0)
#   rehearse4  the same for --config 4, with the gathered-recon check
#   prof       rocprofv3 --kernel-trace --stats of bench.py
#   pmc        the FETCH_SIZE and WRITE_SIZE passes of bench.py (MI355X_MICROARCH.md §HBM)
#   pmc4       the same passes of bench.py --config 4 (BENCH_ARGS: e.g. --levels int32)
#   configs    tools/bench_configs.py (configs 3/4/5 + frame driver)
#   percall    tools/percall.py (drop-in per-call cost); percall_ab: the same over tools/_ab/ (older build)
#   pmc_sq     SQ wave-state pass (issue / wait fractions) of bench.py; CONFIG=4 for the config-4 bench
#   kt_cfg     rocprofv3 kernel trace of tools/bench_configs.py $CONFIGS_ARGS (per-kernel times of configs 3/4/5)
#   rccl       tests/rccl_world1.py (the RCCL branch at world size 1; also in `tests`)
#   valu_rate  tools/ab/_valu_rate: chip-wide issue rate per VALU opcode (build it first, see the .hip)
#   counters   rocprofv3 -L (the counters this box offers)
#   valu_kt / valu_pmc1 / valu_pmc2   the VALU roofline passes over bench_configs $VALU_CFGS
#              (kernel trace; SQ wave/instruction counters; MFMA busy + GRBM clock) -> tools/pmc_valu.py
#   valu_pmc3 / valu_pmc4   instruction counts per unit and per VALU class over the same configs
#              (the measured totals the dynamic mix of tools/valu_dyn.py must reproduce)
#   pmc_cal    tools/ab/_pmc_cal under the pmc3 / pmc4 counter sets: which counter counts which instruction
# pytest selection: PYTEST_K="expr" (passed as -k expr); bench args: BENCH_ARGS="...".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
VALU_CFGS=${VALU_CFGS:-3,4b,5b,closed,closed4}
STEPS=${STEPS:-20}
FRAMES=${FRAMES:-128}
PMC3="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_MFMA SQ_INSTS_VMEM_RD"
PMC4="SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32"
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"

run_step() {
  case "$1" in
    tests)
      echo "== pytest -m gpu"
      timeout -k 10 900 $PT tests -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?
      tail -5 gpurun_out/pytest_gpu_${TAG}.log; return $rc ;;
    smoke)
      echo "== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1; rc=$?
      tail -3 gpurun_out/smoke_${TAG}.log; return $rc ;;
    bench)
      echo "== bench"
      timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 --frames $FRAMES $BENCH_ARGS > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err; rc=$?
      cat gpurun_out/bench_${TAG}.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_${TAG}.err; return $rc ;;
    bench4)
      echo "== bench --config 4"
      timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 $BENCH_ARGS > gpurun_out/bench4_${TAG}.json 2> gpurun_out/bench4_${TAG}.err; rc=$?
      cat gpurun_out/bench4_${TAG}.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench4_${TAG}.err; return $rc ;;
    rehearse2)
      echo "== bench --gpus 2 rehearsal (gloo, one device)"
      NH_DIST_BACKEND=gloo NH_FORCE_DEVICE=0 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --frames 32 $BENCH_ARGS > gpurun_out/rehearse2_${TAG}.json 2> gpurun_out/rehearse2_${TAG}.err; rc=$?
      cat gpurun_out/rehearse2_${TAG}.json; [ $rc -eq 0 ] || tail -20 gpurun_out/rehearse2_${TAG}.err; return $rc ;;
    rehearse4)
      echo "== bench --config 4 --gpus 2 rehearsal (gloo, one device, --check)"
      NH_DIST_BACKEND=gloo NH_FORCE_DEVICE=0 timeout -k 10 400 python bench.py --config 4 --gpus 2 --steps 3 --warmup 1 --frames 4 --check $BENCH_ARGS > gpurun_out/rehearse4_${TAG}.json 2> gpurun_out/rehearse4_${TAG}.err; rc=$?
      cat gpurun_out/rehearse4_${TAG}.json; [ $rc -eq 0 ] || tail -20 gpurun_out/rehearse4_${TAG}.err; return $rc ;;
    prof)
      echo "== rocprof kernel-trace stats"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 bench.py --steps $STEPS --warmup 5 --frames $FRAMES --no-cpu-baseline $BENCH_ARGS > gpurun_out/prof_${TAG}.log 2>&1; rc=$?
      tail -2 gpurun_out/prof_${TAG}.log; return $rc ;;
    pmc)
      echo "== rocprof pmc FETCH_SIZE / WRITE_SIZE"
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_${TAG} -o run -- python3 bench.py --steps 5 --warmup 2 --frames $FRAMES --no-cpu-baseline $BENCH_ARGS > gpurun_out/pmc_fetch_${TAG}.log 2>&1 && \
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_${TAG} -o run -- python3 bench.py --steps 5 --warmup 2 --frames $FRAMES --no-cpu-baseline $BENCH_ARGS > gpurun_out/pmc_write_${TAG}.log 2>&1 ;;
    pmc4)
      echo "== rocprof pmc FETCH_SIZE / WRITE_SIZE of bench.py --config 4 $BENCH_ARGS"
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc4_fetch_${TAG} -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/pmc4_fetch_${TAG}.log 2>&1 && \
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc4_write_${TAG} -o run -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/pmc4_write_${TAG}.log 2>&1 ;;
    configs)
      echo "== bench_configs"
      timeout -k 10 400 python tools/bench_configs.py $CONFIGS_ARGS > gpurun_out/configs_${TAG}.jsonl 2> gpurun_out/configs_${TAG}.err; rc=$?
      cat gpurun_out/configs_${TAG}.jsonl; [ $rc -eq 0 ] || tail -20 gpurun_out/configs_${TAG}.err; return $rc ;;
    percall)
      echo "== per-call cost"
      timeout -k 10 300 python tools/percall.py --phases $PERCALL_ARGS > gpurun_out/percall_${TAG}.json 2> gpurun_out/percall_${TAG}.err; rc=$?
      tail -3 gpurun_out/percall_${TAG}.json; [ $rc -eq 0 ] || tail -20 gpurun_out/percall_${TAG}.err; return $rc ;;
    percall_ab)
      echo "== per-call cost, previous build (tools/_ab/libnanohevc_r01_staging.so)"
      timeout -k 10 300 python tools/percall.py --lib tools/_ab/libnanohevc_r01_staging.so > gpurun_out/percall_r01lib_${TAG}.json 2> gpurun_out/percall_r01lib_${TAG}.err; rc=$?
      tail -3 gpurun_out/percall_r01lib_${TAG}.json; [ $rc -eq 0 ] || tail -20 gpurun_out/percall_r01lib_${TAG}.err; return $rc ;;
    pmc_sq)
      echo "== rocprof pmc SQ wave states (config ${CONFIG:-2})"
      timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_sq_${TAG} -o run -- python3 bench.py --config ${CONFIG:-2} --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/pmc_sq_${TAG}.log 2>&1 ;;
    kt_cfg)
      echo "== rocprof kernel trace of bench_configs $CONFIGS_ARGS"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_cfg_${TAG} -o run -- python3 tools/bench_configs.py $CONFIGS_ARGS > gpurun_out/kt_cfg_${TAG}.log 2>&1 ;;
    rccl)
      echo "== RCCL world-1 gather check"
      timeout -k 10 240 python tests/rccl_world1.py > gpurun_out/rccl_${TAG}.json 2> gpurun_out/rccl_${TAG}.err; rc=$?
      cat gpurun_out/rccl_${TAG}.json; [ $rc -eq 0 ] || tail -20 gpurun_out/rccl_${TAG}.err; return $rc ;;
    valu_rate)
      echo "== VALU issue rates"
      timeout -k 10 120 tools/ab/_valu_rate > gpurun_out/valu_rate_${TAG}.jsonl 2> gpurun_out/valu_rate_${TAG}.err; rc=$?
      tail -3 gpurun_out/valu_rate_${TAG}.jsonl; return $rc ;;
    counters)
      echo "== rocprofv3 -L"
      timeout -s KILL 90 rocprofv3 -L > gpurun_out/counters_${TAG}.txt 2>&1; rc=$?
      grep -c "" gpurun_out/counters_${TAG}.txt; return $rc ;;
    pmc_cal)
      echo "== counter calibration (tools/ab/_pmc_cal)"
      timeout -s KILL 60 rocprofv3 --pmc $PMC3 --output-format csv -d gpurun_out/pmc_cal3_${TAG} -o run -- tools/ab/_pmc_cal > gpurun_out/pmc_cal_${TAG}.log 2>&1 && \
      timeout -s KILL 60 rocprofv3 --pmc $PMC4 --output-format csv -d gpurun_out/pmc_cal4_${TAG} -o run -- tools/ab/_pmc_cal >> gpurun_out/pmc_cal_${TAG}.log 2>&1; rc=$?
      tail -2 gpurun_out/pmc_cal_${TAG}.log; return $rc ;;
    valu_kt|valu_pmc1|valu_pmc2|valu_pmc3|valu_pmc4)
      # one profiler run per config (a config's kernels alone in each CSV)
      for c in ${VALU_CFGS//,/ }; do
        echo "== $1 over bench_configs --configs $c"
        case "$1" in
          valu_kt)   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$1_${TAG}_$c -o run -- python3 tools/bench_configs.py --configs $c --reps 3 > gpurun_out/$1_${TAG}_$c.log 2>&1 || return 1 ;;
          valu_pmc1) timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/$1_${TAG}_$c -o run -- python3 tools/bench_configs.py --configs $c --reps 3 > gpurun_out/$1_${TAG}_$c.log 2>&1 || return 1 ;;
          valu_pmc3) timeout -s KILL 300 rocprofv3 --pmc $PMC3 --output-format csv -d gpurun_out/$1_${TAG}_$c -o run -- python3 tools/bench_configs.py --configs $c --reps 3 > gpurun_out/$1_${TAG}_$c.log 2>&1 || return 1 ;;
          valu_pmc4) timeout -s KILL 300 rocprofv3 --pmc $PMC4 --output-format csv -d gpurun_out/$1_${TAG}_$c -o run -- python3 tools/bench_configs.py --configs $c --reps 3 > gpurun_out/$1_${TAG}_$c.log 2>&1 || return 1 ;;
          valu_pmc2) timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/$1_${TAG}_$c -o run -- python3 tools/bench_configs.py --configs $c --reps 3 > gpurun_out/$1_${TAG}_$c.log 2>&1 || return 1 ;;
        esac
        python3 tools/trim_prof.py gpurun_out/$1_${TAG}_$c
      done ;;
    *)
      echo "unknown step $1"; return 2 ;;
  esac
}

for s in "$@"; do
  run_step "$s" || { echo "== step $s failed (rc=$?); stopping"; exit 1; }
done
echo "== done"
