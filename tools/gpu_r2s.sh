# round-2 session 3: split-K ring fix numerics + HBM-cold decode GEMM A/B, then the full GPU pass
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2s; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_splitk.log python -u -m pytest tests/test_splitk_gpu.py -m gpu -x -v --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
tools/gpu_step.sh 300 $O/dec_hbm.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm.jsonl || exit 1
tools/gpu_step.sh 700 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
tools/gpu_step.sh 300 $O/bench.log python bench.py --steps 3 --warmup 2 --json-out $O/bench.json || exit 1
