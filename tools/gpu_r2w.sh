# decode GEMM: LDS-staged kernel at different workgroup counts (activation re-staging vs parallelism)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2w; mkdir -p $O
for wg in 256 128 64; do
GAI_DEC2_MINWG=$wg tools/gpu_step.sh 200 $O/dec_hbm_$wg.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm_$wg.jsonl || exit 1
done
