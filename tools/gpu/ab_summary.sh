# summary of an ab_tool_step.sh run: the tool's lines matching PATTERN and the step img/s
#   bash tools/gpu/ab_summary.sh TAG PATTERN VAR1 [VAR2 ...]
tag=$1; pat=$2; shift 2
cd "$(dirname "$0")/../../gpurun_out/$tag" || exit 1
for v in base "$@"; do
  for r in 1 2; do
    t=$(grep -h -E "$pat" tool_${v}_$r.log 2>/dev/null | tr '\n' ' ' | cut -c1-200)
    s=$(grep -h '^{' step_${v}_$r.log 2>/dev/null | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)
    echo "== $v $r | $t | $s"
  done
done
