set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/ln
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "layernorm" > gpurun_out/ln/tests.log 2>&1
for v in "" ln512 ln2048; do
  if [ -n "$v" ]; then export VITMI_LIB=$PWD/transformer-stm_amd/build/variants/$v.so; else unset VITMI_LIB; fi
  timeout -k 10 120 python tools/ln_bench.py > gpurun_out/ln/lb_${v:-base}.log 2>&1
done
unset VITMI_LIB
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ln/bench.log 2>&1
