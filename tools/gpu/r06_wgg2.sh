# weight-gradient grouping modes in the C3 / C5 step (VITMI_WGRAD_GROUP 0..3, see vitmi/ops.py), 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_wgg2}
mkdir -p gpurun_out/$tag
for r in 1 2; do
  for v in 0 1 2 3; do
    VITMI_WGRAD_GROUP=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_g${v}_$r.json 2>/dev/null || exit 1
    echo "c3 group=$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_g${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
for v in 0 1 2 3; do
  VITMI_WGRAD_GROUP=$v timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-secondary --no-evidence \
      --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_c5_g${v}.json 2>/dev/null || exit 1
  echo "c5 group=$v $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_c5_g${v}.json'));print(d['value'], d['ms_per_step'])")"
done
