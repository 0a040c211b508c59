# rocprofv3 kernel stats of the bench step: bash tools/gpu/prof.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=${1:-cur}
mkdir -p gpurun_out/prof_$tag
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prof_$tag/prof.log 2>&1
