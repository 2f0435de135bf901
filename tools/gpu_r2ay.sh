# wide-N GEMMs (gate_up) on the part-ring kernel: GEMM / model tests, same-box bench native vs hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2ay; mkdir -p $O
tools/gpu_step.sh 300 $O/pytest.log python -u -m pytest tests/test_gemm_ring_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_splitk_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest.log && ! grep -q "failed" $O/pytest.log || exit 1
tools/gpu_step.sh 300 $O/native.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/native.json || exit 1
GAI_GEMM_POLICY=hipblaslt tools/gpu_step.sh 300 $O/blas.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/blas.json || exit 1
