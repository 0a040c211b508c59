# grouped weight gradients: the new GPU tests, the isolated four-wgrad timing (ViT-B, ViT-L), and the
# C3 / C5 step with the grouped launch vs one launch per problem (VITMI_WGRAD_GROUP=0), 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_wgg}
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 180 --timeout-method thread \
    -k "wgrad" > gpurun_out/$tag/test_ops.log 2>&1 || { tail -30 gpurun_out/$tag/test_ops.log; exit 1; }
tail -2 gpurun_out/$tag/test_ops.log
for c in b l; do timeout -k 10 120 python3 tools/wgrad_group_bench.py $c 2>&1 | grep -v amdgpu.ids || exit 1; done
for r in 1 2; do
  for v in 1 0; do
    VITMI_WGRAD_GROUP=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_g${v}_$r.json 2>/dev/null || exit 1
    echo "c3 group=$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_g${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
for v in 1 0; do
  VITMI_WGRAD_GROUP=$v timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-secondary --no-evidence \
      --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_c5_g${v}.json 2>/dev/null || exit 1
  echo "c5 group=$v $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_c5_g${v}.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/$tag/test_all.log 2>&1; tail -3 gpurun_out/$tag/test_all.log
