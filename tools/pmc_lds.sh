set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_lds; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
C2="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --configs none --secondary= --alt-streams 0"
i=0
for G in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE" "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/pmc/p$i -o run -- $C2 > $O/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $O/p$i.log; exit 1; }
done
cd $R && python3 tools/prof_stages.py $O --skip 6 --take 20 --out $O/stages.json > $O/stages.txt && cat $O/stages.txt
