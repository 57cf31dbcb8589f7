R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH -d $R/gpurun_out/rfA -o run -- python3 $R/tools/_diag_refill.py > $R/gpurun_out/rfA.log 2>&1 &&
$P --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_ANY -d $R/gpurun_out/rfB -o run -- python3 $R/tools/_diag_refill.py > $R/gpurun_out/rfB.log 2>&1
echo rc=$?
