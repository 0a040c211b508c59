#!/bin/bash
# side-by-side report of tools/gpu/ab_var.sh output: bash tools/abv_report.sh v1 v2 ...
cd "$(dirname "$0")/../gpurun_out/abv"
files="gb_base.log"; for v in "$@"; do files="$files gb_$v.log"; done
paste $files | grep -v amdgpu.ids | python3 -c "
import sys,re
for line in sys.stdin:
    cols=line.rstrip('\n').split('\t')
    name=cols[0].split(':')[0]
    vals=[re.findall(r'([0-9.]+) TFLOP',c) for c in cols]
    print(f'{name:30s}', '  '.join(f'{v[0]:>7s}' if v else '   -   ' for v in vals))
"
grep -o '"value": [0-9.]*' bench_base.log $(for v in "$@"; do echo bench_$v.log; done)
