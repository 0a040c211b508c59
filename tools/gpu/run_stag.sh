set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stag
for r in 1 2; do
for cfg in "0 0" "3 0" "4 1" "2 2"; do
  set -- $cfg
  timeout -k 10 300 python3 tools/bench_exp.py $1 $2 --no-cpu-baseline --no-evidence --steps 10 --warmup 3 > gpurun_out/stag/b_$1_$2_$r.log 2>&1 || exit 1
done
done
