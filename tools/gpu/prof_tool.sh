# per-kernel rocprofv3 summary of a short bench run, for ab_tool_step.sh (the library under test
# comes from VITMI_LIB); prints the summary lines matching PATTERN
#   bash tools/gpu/prof_tool.sh TAG PATTERN
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
d=$PWD/gpurun_out/$1/prof_$(basename "${VITMI_LIB:-base}" .so)_$$
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-evidence --no-secondary --steps 5 --warmup 2 > /dev/null 2>&1 || exit 1
python3 tools/prof_summary.py "$(find $d -name 'run_kernel_stats.csv' | head -1)" 7 > $d.txt || exit 1
grep -E "$2" $d.txt
rm -rf $d
