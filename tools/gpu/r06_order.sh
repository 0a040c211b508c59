# backward kernel order inside a block (VITMI_BWD_ORDER bits: 1 = fc1 dgrad before the MLP weight
# gradients, 2 = the grouped attention-pair weight gradients before the qkv dgrad): C3 step, 2 rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
tag=${1:-r06_order}
mkdir -p gpurun_out/$tag
for r in 1 2; do
  for v in 0 1 2 3; do
    VITMI_BWD_ORDER=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence \
        --no-cpu-baseline --no-parity > gpurun_out/$tag/bench_o${v}_$r.json 2>/dev/null || exit 1
    echo "c3 order=$v $r $(python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench_o${v}_$r.json'));print(d['value'], d['ms_per_step'], d['phases_ms']['backward'])")"
  done
done
