set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2t; mkdir -p $O
tools/gpu_step.sh 300 $O/dec_hbm.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm.jsonl || exit 1
tools/gpu_step.sh 700 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
