# counter passes: full-line prefill GEMM kernels vs hipBLASLt (O and down projection shapes)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_gemm.sh 4096 4096 gpurun_out/pmc_o w4p w4d w4r blas || exit 1
bash tools/pmc_gemm.sh 4096 14336 gpurun_out/pmc_down w4d w4r blas || exit 1
