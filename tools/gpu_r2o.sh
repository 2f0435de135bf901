# fp8 KV kernels + sampler fast path: new GPU tests, sampler timing, headline bench with fp8 KV (option)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2o; mkdir -p $O
tools/gpu_step.sh 400 $O/pytest_new.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "sample or prefill or decode or rope" || exit 1
tools/gpu_step.sh 120 $O/sample_bench.log python tools/sample_bench.py || exit 1
tools/gpu_step.sh 400 $O/bench_fp8kv.log python bench.py --steps 3 --warmup 2 --no-probes --kv-cache-dtype fp8 --json-out $O/bench_fp8kv.json || exit 1
tools/gpu_step.sh 400 $O/bench_bf16.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench_bf16.json || exit 1
