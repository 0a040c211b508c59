# alternating step A/B of an environment switch: bash tools/gpu/env_ab2.sh TAG VAR VALUE_A VALUE_B [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tag=$1; var=$2; a=$3; b=$4; n=${5:-3}
mkdir -p gpurun_out/$tag
for r in $(seq 1 $n); do
  for v in $a $b; do
    env $var=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 20 --warmup 3 > gpurun_out/$tag/${v}_$r.json 2> gpurun_out/$tag/${v}_$r.err || exit 1
    echo "$var=$v round $r: $(python3 -c "import json; d=json.load(open('gpurun_out/$tag/${v}_$r.json')); print(d['value'], d['ms_per_step'])")"
  done
done
