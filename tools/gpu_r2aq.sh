# full-line double-unit prefill GEMM: numerics, A/B vs hipBLASLt, headline bench auto vs native policy
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2aq; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_ring.log python -u -m pytest tests/test_gemm_ring_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_ring.log && ! grep -q "failed" $O/pytest_ring.log || exit 1
tools/gpu_step.sh 200 $O/gemm_bench.log python -u tools/gemm_bench.py --rounds 5 --out $O/gemm_w4r.jsonl || exit 1
tools/gpu_step.sh 300 $O/bench_auto.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench_auto.json || exit 1
GAI_GEMM_POLICY=native tools/gpu_step.sh 300 $O/bench_native.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench_native.json || exit 1
