# deep-K decode GEMM (down) on the LDS-staged kernel with K-split slabs: numerics + HBM A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2ag; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_splitk.log python -u -m pytest tests/test_splitk_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_splitk.log && ! grep -q "failed" $O/pytest_splitk.log || exit 1
tools/gpu_step.sh 300 $O/dec_hbm.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm.jsonl || exit 1
