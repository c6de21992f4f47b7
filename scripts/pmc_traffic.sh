#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs) over a probe driver; summary JSON via pmc_summary.py.
# usage: OUT=<dir> KREGEX=<regex> PROBE=<script in scripts/> scripts/pmc_traffic.sh
set -o pipefail
cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-pmct}
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "${KREGEX:-k_}" --output-format csv -d $O/$c -o run -- \
    python3 $R/scripts/${PROBE:-pmc_probe.py} > $O/$c.log 2>&1 || { echo "pass $c failed"; tail -5 $O/$c.log; exit 1; }
done
F=$(find $O/FETCH_SIZE -name "*counter_collection.csv" | head -1)
W=$(find $O/WRITE_SIZE -name "*counter_collection.csv" | head -1)
python3 $R/scripts/pmc_summary.py "$F" "$W" $O/traffic.json && cat $O/traffic.json
