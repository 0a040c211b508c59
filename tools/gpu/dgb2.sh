set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/dgb2
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread -k "fused_bias or model or block or mlp" > gpurun_out/dgb2/tests.log 2>&1
for r in 1 2; do
for F in 0 1; do
  echo "== F $F" >> gpurun_out/dgb2/bench.txt
  VITMI_FUSED_BIAS=$F timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/dgb2/bench.txt 2>&1
done
done
