# same-box GEMM policy A/B after the fused prefill RoPE epilogue + final headline kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2ax; mkdir -p $O
tools/gpu_step.sh 300 $O/native1.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/native1.json || exit 1
GAI_GEMM_POLICY=hipblaslt tools/gpu_step.sh 300 $O/blas.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/blas.json || exit 1
tools/gpu_step.sh 300 $O/native2.log python bench.py --steps 4 --warmup 2 --no-probes --json-out $O/native2.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_fin -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-probes > $O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/rocprof_summary.py "/tmp/prof_fin/**/*kernel_stats.csv" -o $O/stats_final.csv --top 40 > /dev/null 2>&1
