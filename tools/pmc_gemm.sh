# rocprofv3 counter passes of one prefill GEMM shape: hand-written kernels vs hipBLASLt.
# usage: tools/pmc_gemm.sh N K OUTDIR ARM...   (e.g. 4096 4096 gpurun_out/pmc_o w4d w4r blas)
# PMC_DRIVER=attn_one.py: the same passes over the headline prefill-attention chunk (arms hl1 / hl2)
set -o pipefail
N=$1; K=$2; OD=$3; shift 3
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/$OD
mkdir -p $O
DRV=${PMC_DRIVER:-gemm_one.py}
for arm in "$@"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/t_$arm -o t --output-format csv -- python3 $R/tools/$DRV $arm $N $K > $O/t_$arm.log 2>&1 || exit 2
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -d $O/p1_$arm -o p1 --output-format csv -- python3 $R/tools/$DRV $arm $N $K > $O/p1_$arm.log 2>&1 || exit 3
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM -d $O/p2_$arm -o p2 --output-format csv -- python3 $R/tools/$DRV $arm $N $K > $O/p2_$arm.log 2>&1 || exit 4
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d $O/p3_$arm -o p3 --output-format csv -- python3 $R/tools/$DRV $arm $N $K > $O/p3_$arm.log 2>&1 || exit 5
done
echo ok
