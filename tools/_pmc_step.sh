R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $R/gpurun_out/pmcA -o run -- python3 $R/tools/_diag_pmc.py > $R/gpurun_out/pmcA.log 2>&1 &&
$P --pmc FETCH_SIZE -d $R/gpurun_out/pmcB -o run -- python3 $R/tools/_diag_pmc.py > $R/gpurun_out/pmcB.log 2>&1 &&
$P --pmc WRITE_SIZE -d $R/gpurun_out/pmcC -o run -- python3 $R/tools/_diag_pmc.py > $R/gpurun_out/pmcC.log 2>&1 &&
$P --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcD -o run -- python3 $R/tools/_diag_pmc.py > $R/gpurun_out/pmcD.log 2>&1
echo rc=$?
