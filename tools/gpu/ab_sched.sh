# A/B of the gemm256 K-loop schedules (VITMI_GEMM_SCHED 1 = staggered, 0 = lockstep)
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "linear or gemm" > gpurun_out/ab/tests_ops.log 2>&1
VITMI_GEMM_SCHED=0 timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/ab/gb_s0.log 2>&1
VITMI_GEMM_SCHED=1 timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/ab/gb_s1.log 2>&1
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests_all.log 2>&1
VITMI_GEMM_SCHED=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab/bench_s0.log 2>&1
VITMI_GEMM_SCHED=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab/bench_s1.log 2>&1
