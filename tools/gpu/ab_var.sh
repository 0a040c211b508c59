# A/B of compiled variants (tools/build_variant.sh) against the in-tree library: GEMM
# microbench + quick bench per variant.  usage: bash tools/gpu/ab_var.sh v1 v2 ...
set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/abv
timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/abv/gb_base.log 2>&1
for v in "$@"; do
  VITMI_LIB=$PWD/transformer-stm_amd/build/variants/$v.so timeout -k 10 200 python tools/gemm_bench.py 20 > gpurun_out/abv/gb_$v.log 2>&1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/abv/bench_base.log 2>&1
for v in "$@"; do
  VITMI_LIB=$PWD/transformer-stm_amd/build/variants/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/abv/bench_$v.log 2>&1
done
