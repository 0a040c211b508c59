# non-temporal stores in the LayerNorm kernels (ln1) and in Adam (ad1) against the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in ln1 ad1; do
  VITMI_LIB=$PWD/transformer-stm_amd/variants/$v.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -k "layernorm or optim or adam or vit_b" -x -q --timeout 120 --timeout-method thread > gpurun_out/ntmisc_test_$v.log 2>&1 || exit 1
done
bash tools/gpu/kab.sh ntmisc "layernorm or optim" "python3 tools/ln_bench.py" ln1 ad1
