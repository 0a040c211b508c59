# C5 (ViT-L/16 384 px bs 64) with the side-stream weight gradients: grouping modes 3 (default) / 2 / 0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_c5g}
mkdir -p gpurun_out/$tag
for r in 1 2; do
  for v in 3 2 0; do
    VITMI_WGRAD_GROUP=$v timeout -k 10 300 python3 bench.py --config c5 --steps 6 --warmup 2 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_g${v}_$r.json 2>/dev/null || exit 1
    echo "c5 group=$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_g${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['backward'])")"
  done
done
