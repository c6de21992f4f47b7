#!/bin/bash
# rocprofv3 --kernel-trace --stats of one bench config (1 warm-up + N timed steps); summary CSVs land
# in gpurun_out/trace_<config>/. usage: scripts/trace_config.sh <config> [steps] [extra bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-c2}; STEPS=${2:-2}; shift; shift
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/trace_$CFG
cd /tmp && exec rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_$CFG -o run -- \
  python3 $R/bench.py --config $CFG --steps $STEPS --warmup 1 --cpu-baseline off --pmc off --extras off "$@"
