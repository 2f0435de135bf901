# QKV / O (K = 4096) on the LDS-staged K-split kernel too? A/B by GAI_DEC2_PART_MINK
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2ai; mkdir -p $O
GAI_DEC2_PART_MINK=4096 tools/gpu_step.sh 200 $O/pytest_splitk.log python -u -m pytest tests/test_splitk_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_splitk.log && ! grep -q "failed" $O/pytest_splitk.log || exit 1
GAI_DEC2_PART_MINK=4096 tools/gpu_step.sh 300 $O/dec_hbm_4096.log python -u tools/kernel_bench.py --only dec_hbm --out $O/dec_hbm_4096.jsonl || exit 1
GAI_DEC2_PART_MINK=4096 tools/gpu_step.sh 400 $O/bench_4096.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench_4096.json || exit 1
tools/gpu_step.sh 400 $O/bench_default.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench_default.json || exit 1
