# MLP weight-gradient order (VITMI_MLP_WG_REV=1: fc1's, which reads the du DGELU just wrote, first)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_mlprev}
mkdir -p gpurun_out/$tag
for r in 1 2 3; do
  for v in 0 1; do
    VITMI_MLP_WG_REV=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_r${v}_$r.json 2>/dev/null || exit 1
    echo "c3 rev=$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_r${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['backward'])")"
  done
done
