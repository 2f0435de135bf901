# prefill attention: longest-tile-first order; kernel bench, counters, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2aa; mkdir -p $O
tools/gpu_step.sh 200 $O/pytest_attn.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "prefill or attention" --timeout 100 --timeout-method thread -p no:cacheprovider || exit 1
tools/gpu_step.sh 200 $O/kb_prefill.log python -u tools/kernel_bench.py --only prefill --out $O/kb_prefill.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -d $O/pmc1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --only prefill > $O/pmc1.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d $O/pmc2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --only prefill > $O/pmc2.log 2>&1 || exit 4
cd $GRAFT_REPO_ROOT
tools/gpu_step.sh 300 $O/bench.log python bench.py --steps 3 --warmup 2 --no-probes --json-out $O/bench.json || exit 1
