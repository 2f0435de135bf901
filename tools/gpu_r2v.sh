# LDS-staged decode GEMM: numerics, HBM-cold A/B vs split-K (psw) and hipBLASLt, then the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2v; mkdir -p $O
tools/gpu_step.sh 240 $O/pytest_splitk.log python -u -m pytest tests/test_splitk_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_splitk.log && ! grep -q "failed" $O/pytest_splitk.log || exit 1
tools/gpu_step.sh 300 $O/dec_hbm.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm.jsonl || exit 1
tools/gpu_step.sh 300 $O/bench.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench.json || exit 1
