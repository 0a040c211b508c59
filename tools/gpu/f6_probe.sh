# FP6-rate probe: the bf16f8 forward GEMMs with their correction MFMAs issued as e2m3 (variant
# f6time, results meaningless) against the in-tree e4m3 build, isolated GEMMs and the C3 bf16f8 step.
#   bash tools/gpu/f6_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=${1:-f6probe}
mkdir -p gpurun_out/$tag
V=$PWD/transformer-stm_amd/variants/f6time.so
for round in 1 2; do
  timeout -k 10 120 python3 tools/f8_shapes.py > gpurun_out/$tag/shapes_base_$round.txt 2>&1 || exit 1
  VITMI_LIB=$V timeout -k 10 120 python3 tools/f8_shapes.py > gpurun_out/$tag/shapes_f6_$round.txt 2>&1 || exit 1
  timeout -k 10 200 python3 bench.py --dtype bf16f8 --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
      > gpurun_out/$tag/bench_base_$round.json 2> gpurun_out/$tag/bench_base_$round.err || exit 1
  VITMI_LIB=$V timeout -k 10 200 python3 bench.py --dtype bf16f8 --steps 10 --warmup 3 --no-secondary --no-evidence \
      --no-cpu-baseline > gpurun_out/$tag/bench_f6_$round.json 2> gpurun_out/$tag/bench_f6_$round.err || exit 1
done
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-secondary --no-evidence --no-cpu-baseline \
    > gpurun_out/$tag/bench_bf16.json 2> gpurun_out/$tag/bench_bf16.err || exit 1
for f in gpurun_out/$tag/shapes_*; do echo "== $f"; cat $f; done
for f in gpurun_out/$tag/bench_*.json; do echo "== $f"; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['phases_ms'])"; done
