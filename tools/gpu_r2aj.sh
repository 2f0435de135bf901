# add+RMSNorm decode tail: 1024-thread x 4-column variant vs 256 x 8 (A/B in kernel profiles)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2aj; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_splitk.log python -u -m pytest tests/test_splitk_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_splitk.log && ! grep -q "failed" $O/pytest_splitk.log || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_w4 -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-probes > $GRAFT_REPO_ROOT/$O/prof_w4.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/rocprof_summary.py "/tmp/prof_w4/**/*kernel_stats.csv" -o $O/stats_w4.csv --top 40 > /dev/null 2>&1
