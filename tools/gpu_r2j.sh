# round-2 GPU pass: gpu tests, prefill GEMM A/B, headline bench (native GEMM policy vs tune), kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2k; mkdir -p $O
tools/gpu_step.sh 500 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
tools/gpu_step.sh 300 $O/gemm_bench.log python tools/gemm_bench.py --rounds 5 --out $O/gemm_ring.jsonl || exit 1
tools/gpu_step.sh 240 $O/bench_native.log python bench.py --steps 3 --warmup 2 --json-out $O/bench_native.json || exit 1
GAI_GEMM_POLICY=tune tools/gpu_step.sh 240 $O/bench_tune.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench_tune.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-probes > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/rocprof_summary.py "/tmp/prof/**/*kernel_stats.csv" -o $O/bench_native_kernel_stats.csv --top 40 > $O/prof_summary.txt 2>&1
