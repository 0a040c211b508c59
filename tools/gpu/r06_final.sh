# Round 6 evidence: the bench line (evidence legs + secondary lines, as the driver runs it) and a
# rocprofv3 kernel summary of the same step (tools/gpu/bench.sh), then the attention kernels' counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag=${1:-r06_final}
bash tools/gpu/bench.sh $tag --steps 20 --warmup 5 || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/$tag/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d['parity']['logits_max_abs']); [print(k, v.get('value'), v.get('parity', {}).get('logits_max_abs')) for k, v in d.get('secondary', {}).items()]"
head -26 gpurun_out/$tag/summary.txt
bash tools/gpu/attn_pmc.sh ${tag}_attn_pmc || exit 1
cat gpurun_out/${tag}_attn_pmc/table.txt
