# final tree: full GPU tier + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2az; mkdir -p $O
tools/gpu_step.sh 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || exit 1
tools/gpu_step.sh 200 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
