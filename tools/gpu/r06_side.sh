# weight gradients on a side stream (VITMI_WGRAD_STREAM=1) filling the dgrad chain's launch tails,
# against the current stream: model tests under the switch, the C3 / C5 step, 2-3 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_side}
mkdir -p gpurun_out/$tag
VITMI_WGRAD_STREAM=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_autograd.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || { tail -30 gpurun_out/$tag/test.log; exit 1; }
tail -1 gpurun_out/$tag/test.log
for r in 1 2 3; do
  for v in 0 1; do
    VITMI_WGRAD_STREAM=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_s${v}_$r.json 2>/dev/null || exit 1
    echo "c3 side=$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_s${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['backward'])")"
  done
done
for v in 0 1; do
  VITMI_WGRAD_STREAM=$v timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-secondary --no-evidence \
      --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_c5_s${v}.json 2>/dev/null || exit 1
  echo "c5 side=$v $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_c5_s${v}.json'));print(d['value'], d['ms_per_step'])")"
done
