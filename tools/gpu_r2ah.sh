# single weight layout (no fragment-shuffled copies): tests, bench, profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2ah; mkdir -p $O
tools/gpu_step.sh 600 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || exit 1
tools/gpu_step.sh 400 $O/bench.log python bench.py --steps 5 --warmup 2 --json-out $O/bench.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-probes > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/rocprof_summary.py "/tmp/prof/**/*kernel_stats.csv" -o $O/bench_kernel_stats.csv --top 50 > $O/prof_summary.txt 2>&1
