# Decode-step HBM traffic per kernel (Llama-3-8B, batch 64, ctx 2535, eager forwards): a kernel-trace pass for the
# durations, then FETCH_SIZE and WRITE_SIZE in runs of their own (3 + 2 TCC counters: one run holds at most 4).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5pmcd
mkdir -p $O
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o t -- python3 $R/tools/decode_kernels.py --batch 64 --ctx 2535 --iters 5 > $O/t.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p -o p -- python3 $R/tools/decode_kernels.py --batch 64 --ctx 2535 --iters 5 > $O/p.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o w -- python3 $R/tools/decode_kernels.py --batch 64 --ctx 2535 --iters 5 > $O/w.log 2>&1 || exit 4
echo ok
