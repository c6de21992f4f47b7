#!/bin/bash
# rocprofv3 --kernel-trace --stats of one bench config (1 warm-up + N timed steps). Keeps the
# per-kernel stats CSV and a steady-state window summary (scripts/trace_window.py) in
# gpurun_out/trace_<config>/ and deletes the (large) raw kernel trace.
# usage: scripts/trace_config.sh <config> [steps] [window_ms] [extra bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-c2}; STEPS=${2:-2}; WIN=${3:-300}; shift 3
export TMPDIR=/tmp
O=$R/gpurun_out/trace_$CFG
mkdir -p $O
cd /tmp || exit 1
rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/trace_$CFG -o run -- \
  python3 $R/bench.py --config $CFG --steps $STEPS --warmup 1 --cpu-baseline off --pmc off --extras off "$@" \
  > $O/bench.log 2>&1
rc=$?
KT=$(find /tmp/trace_$CFG -name "*kernel_trace.csv" | head -1)
KS=$(find /tmp/trace_$CFG -name "*kernel_stats.csv" | head -1)
[ -n "$KS" ] && cp "$KS" $O/kernel_stats.csv
[ -n "$KT" ] && python3 $R/scripts/trace_window.py "$KT" $WIN $O/kernel_stats_window.csv > $O/window.txt
[ -n "$KT" ] && python3 $R/scripts/trace_gaps.py "$KT" $WIN > $O/gaps.txt
rm -rf /tmp/trace_$CFG
tail -3 $O/bench.log
exit $rc
