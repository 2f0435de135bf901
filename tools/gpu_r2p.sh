# sampler single-pass fast path: sampling tests + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2p; mkdir -p $O
tools/gpu_step.sh 300 $O/pytest_sample.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "sample" || exit 1
tools/gpu_step.sh 120 $O/sample_bench.log python tools/sample_bench.py || exit 1
