# Round 5: C4 fused kernels on CU-partitioned streams (tools/exp_cupart.py) -> gpurun_out/cup
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/cup
KGX_LIB=keras-geometric_amd/lib/variants/libkgx_cupart.so timeout -k 10 400 python -u tools/exp_cupart.py > gpurun_out/cup/cupart.json 2> gpurun_out/cup/cupart.err
