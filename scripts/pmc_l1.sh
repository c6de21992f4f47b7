# SQ / GRBM counter passes (two runs, within the per-pass block limits) over a probe script, summed
# per kernel by scripts/pmc_sq.py.
# usage: [PROBE=pmc_probe_l1.py] [KREGEX=k_plane] [OUT=pmcl1] bash scripts/pmc_l1.sh
set -o pipefail
cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PROBE=${PROBE:-pmc_probe_l1.py}; KREGEX=${KREGEX:-k_plane}; OUT=${OUT:-pmcl1}
mkdir -p $R/gpurun_out/$OUT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "$KREGEX" --output-format csv -d $R/gpurun_out/$OUT/p$i -o run -- python3 $R/scripts/$PROBE > $R/gpurun_out/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/$OUT/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_sq.py $R/gpurun_out/$OUT
