# padded-EP graph capture (custom AR tests passed in the previous call)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2q; mkdir -p $O
tools/gpu_step.sh 150 $O/pytest_moe.log python -u -m pytest tests/test_moe_gpu.py -m gpu -x -v --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
