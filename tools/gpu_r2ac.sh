# (1) prefill attention softmax/PV interleave; (2) legacy split-K workgroup-count sweep for QKV / O
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2ac; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_attn.log python -u -m pytest tests/test_kernels_gpu.py tests/test_context_parallel_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_attn.log && ! grep -q "failed" $O/pytest_attn.log || exit 1
tools/gpu_step.sh 200 $O/kb_prefill.log python -u tools/kernel_bench.py --only prefill --out $O/kb_prefill.jsonl || exit 1
for wg in 512 256 128 1024; do
GAI_SPLITK_LEGACY_MINWG=$wg tools/gpu_step.sh 200 $O/dec_hbm_$wg.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm_$wg.jsonl || exit 1
done
tools/gpu_step.sh 300 $O/bench.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench.json || exit 1
