# slice-staging split-K kernel: 8 vs 4 waves per workgroup (QKV / O at decode), then bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2y; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_splitk.log python -u -m pytest tests/test_splitk_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
for w in 8 4; do
GAI_SPLITK_WPG=$w tools/gpu_step.sh 200 $O/dec_hbm_wpg$w.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm_wpg$w.jsonl || exit 1
done
tools/gpu_step.sh 300 $O/bench.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench.json || exit 1
