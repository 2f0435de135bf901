# native GEMM policy by default: full GPU tier, headline bench, kernel profile (expect no Cijk_* kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2ar; mkdir -p $O
tools/gpu_step.sh 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || exit 1
tools/gpu_step.sh 400 $O/bench.log python bench.py --steps 5 --warmup 2 --json-out $O/bench.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_nat -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-probes > $O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/rocprof_summary.py "/tmp/prof_nat/**/*kernel_stats.csv" -o $O/stats_native.csv --top 40 > /dev/null 2>&1
