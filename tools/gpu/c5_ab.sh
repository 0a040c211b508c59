set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -k "attention or attn" -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/test.log 2>&1 || exit 1
for round in 1 2; do
for v in base "$@"; do
  lib=""; [ $v != base ] && lib=$PWD/transformer-stm_amd/variants/$v.so
  VITMI_LIB=$lib timeout -k 10 120 python3 tools/attn_bench.py 64 577 16 > gpurun_out/$tag/attn_${v}_$round.log 2>&1 || exit 1
done
done
for v in base "$@"; do
  lib=""; [ $v != base ] && lib=$PWD/transformer-stm_amd/variants/$v.so
  VITMI_LIB=$lib timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-evidence --steps 6 --warmup 2 > gpurun_out/$tag/c5_$v.log 2>&1 || exit 1
done
