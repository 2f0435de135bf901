# headline bench under both GEMM policies + kernel profile of the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2u; mkdir -p $O
GAI_GEMM_POLICY=native tools/gpu_step.sh 300 $O/bench_native.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench_native.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-probes > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/rocprof_summary.py "/tmp/prof/**/*kernel_stats.csv" -o $O/bench_kernel_stats.csv --top 40 > $O/prof_summary.txt 2>&1
