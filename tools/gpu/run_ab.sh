# GPU tests of the GEMM/model path, then an A/B of the step time against the variants named
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_test.log 2>&1 || exit 1
bash tools/gpu/ab.sh $tag "python3 bench.py --no-cpu-baseline --no-evidence --steps 10 --warmup 3" "$@"
