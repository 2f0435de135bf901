# round-2 re-entry check: full GPU test tier, smoke, persistent GEMM A/B, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2an; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_ring.log python -u -m pytest tests/test_gemm_ring_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_ring.log && ! grep -q "failed" $O/pytest_ring.log || exit 1
tools/gpu_step.sh 200 $O/gemm_bench.log python -u tools/gemm_bench.py --rounds 5 --out $O/gemm_w4p.jsonl || exit 1
tools/gpu_step.sh 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || exit 1
tools/gpu_step.sh 200 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh 400 $O/bench.log python bench.py --steps 5 --warmup 2 --json-out $O/bench.json || exit 1
