# split-K variant sweep (legacy slice-staging vs register-streamed) on the narrow decode projections
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2ad; mkdir -p $O
for v in 1 2; do
GAI_SPLITK_V=$v tools/gpu_step.sh 200 $O/dec_hbm_v$v.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm_v$v.jsonl || exit 1
done
