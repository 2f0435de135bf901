# final round-2 check of the committed tree: full GPU tier, smoke, 10-step headline bench,
# DP2 and TP2 single-GPU rehearsals of the driver's multi-GPU runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2au; mkdir -p $O
tools/gpu_step.sh 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || exit 1
tools/gpu_step.sh 200 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh 500 $O/bench.log python bench.py --steps 10 --warmup 3 --json-out $O/bench.json || exit 1
GAI_SINGLE_DEVICE=1 tools/gpu_step.sh 400 $O/dp2_rehearsal.log python bench.py --gpus 2 --steps 2 --warmup 1 --no-probes || exit 1
GAI_SINGLE_DEVICE=1 tools/gpu_step.sh 300 $O/tp2_rehearsal.log python bench.py --gpus 2 --config 3 --rag70b-model tiny --steps 2 --warmup 1 || exit 1
