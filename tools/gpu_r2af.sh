# round-2 evidence pass: full GPU tests, DP=2 and TP=2 single-GPU rehearsals, headline bench (20 steps), kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r2af; mkdir -p $O
tools/gpu_step.sh 600 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
GAI_SINGLE_DEVICE=1 tools/gpu_step.sh 400 $O/dp2_rehearsal.log python bench.py --gpus 2 --steps 2 --warmup 1 --no-probes || exit 1
GAI_SINGLE_DEVICE=1 tools/gpu_step.sh 300 $O/tp2_rehearsal.log python bench.py --gpus 2 --config 3 --rag70b-model tiny --steps 2 --warmup 1 || exit 1
tools/gpu_step.sh 400 $O/bench.log python bench.py --steps 10 --warmup 3 --json-out $O/bench.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-probes > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/rocprof_summary.py "/tmp/prof/**/*kernel_stats.csv" -o $O/bench_kernel_stats.csv --top 50 > $O/prof_summary.txt 2>&1
