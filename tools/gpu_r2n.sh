# sampler timing (new vs old path via flat rows), single-GPU TP rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2n; mkdir -p $O
tools/gpu_step.sh 120 $O/sample_bench.log python tools/sample_bench.py || exit 1
GAI_SINGLE_DEVICE=1 tools/gpu_step.sh 300 $O/tp2_rehearsal.log python bench.py --gpus 2 --config 3 --rag70b-model tiny --steps 2 --warmup 1 || exit 1
