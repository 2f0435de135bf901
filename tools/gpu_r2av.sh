# same-box A/B of the GEMM policy on the headline bench: native (default) / hipblaslt / native
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2av; mkdir -p $O
tools/gpu_step.sh 300 $O/native1.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/native1.json || exit 1
GAI_GEMM_POLICY=hipblaslt tools/gpu_step.sh 300 $O/blas.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/blas.json || exit 1
tools/gpu_step.sh 300 $O/native2.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/native2.json || exit 1
