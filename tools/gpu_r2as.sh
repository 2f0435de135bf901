# K-based prefill kernel rule (w4d for K < 8192, w4r for deep K): GEMM tests, A/B, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2as; mkdir -p $O
tools/gpu_step.sh 300 $O/pytest_gemm.log python -u -m pytest tests/test_gemm_ring_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_gemm.log && ! grep -q "failed" $O/pytest_gemm.log || exit 1
tools/gpu_step.sh 200 $O/gemm_bench.log python -u tools/gemm_bench.py --rounds 5 --out $O/gemm_rule.jsonl || exit 1
tools/gpu_step.sh 400 $O/bench.log python bench.py --steps 5 --warmup 2 --json-out $O/bench.json || exit 1
