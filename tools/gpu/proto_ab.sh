set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/proto1
timeout -k 10 300 python3 tools/proto/bench_proto.py 20 > gpurun_out/proto1/bench_proto.txt 2>&1
