# prefill QKV GEMM with fused RoPE + paged KV write: numerics, model tests, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2aw; mkdir -p $O
tools/gpu_step.sh 300 $O/pytest_fused.log python -u -m pytest tests/test_gemm_ring_gpu.py -k "rope_kv or w4d" tests/test_models_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_fused.log && ! grep -q "failed" $O/pytest_fused.log || exit 1
tools/gpu_step.sh 300 $O/bench_fused.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/bench_fused.json || exit 1
GAI_FUSE_ROPE=0 tools/gpu_step.sh 300 $O/bench_unfused.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/bench_unfused.json || exit 1
tools/gpu_step.sh 600 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
