set -o pipefail
cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/${OUT:-pmcp}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_FLAT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "${KREGEX:-k_plane}" --output-format csv -d $R/gpurun_out/${OUT:-pmcp}/p$i -o run -- python3 $R/scripts/${PROBE:-pmc_probe.py} > $R/gpurun_out/${OUT:-pmcp}/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/${OUT:-pmcp}/p$i.log; exit 1; }
done
echo ok
