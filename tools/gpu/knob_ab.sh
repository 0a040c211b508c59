# A/B of a knob variant (variants/$2.so) against the in-tree build: C3 --dtype $3 bench lines,
# alternating.   bash tools/gpu/knob_ab.sh TAG VARIANT DTYPE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1; var=$2; dt=${3:-bf16f8}
mkdir -p gpurun_out/$tag
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --config c3 --dtype $dt --steps 5 --warmup 2 --no-secondary --no-evidence \
      --no-cpu-baseline > gpurun_out/$tag/base$i.json 2>/dev/null || exit 1
  VITMI_LIB=$PWD/transformer-stm_amd/variants/$var.so timeout -k 10 300 python3 bench.py --config c3 --dtype $dt \
      --steps 5 --warmup 2 --no-secondary --no-evidence --no-cpu-baseline > gpurun_out/$tag/var$i.json 2>/dev/null || exit 1
done
grep -Ho '"value": [0-9.]*' gpurun_out/$tag/*.json
