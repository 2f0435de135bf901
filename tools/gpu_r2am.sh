# prefill attention: scalar block-table lookups, buffer-load staging, no Q-load wait merge in the loop
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2am; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_attn.log python -u -m pytest tests/test_kernels_gpu.py tests/test_context_parallel_gpu.py tests/test_model_families_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_attn.log && ! grep -q "failed" $O/pytest_attn.log || exit 1
tools/gpu_step.sh 200 $O/kb_prefill.log python -u tools/kernel_bench.py --only prefill --out $O/kb_prefill.jsonl || exit 1
tools/gpu_step.sh 300 $O/bench.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench.json || exit 1
