# with the weight gradients on the side stream: the grouping modes again (VITMI_WGRAD_GROUP 0 / 1 / 3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_side2}
mkdir -p gpurun_out/$tag
for r in 1 2; do
  for v in 3 0 1; do
    VITMI_WGRAD_GROUP=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_g${v}_$r.json 2>/dev/null || exit 1
    echo "c3 group=$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_g${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['backward'])")"
  done
done
