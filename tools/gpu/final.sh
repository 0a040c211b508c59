# round-end rehearsal: full GPU suite, smoke, default bench (with cpu_baseline), kernel stats
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/final/bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/final/prof.log 2>&1
