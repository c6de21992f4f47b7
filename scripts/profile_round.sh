#!/bin/bash
# One round's profiling evidence, written to gpurun_out/<tag>/ (copy what is judged into profiles/):
#   kbench.log          per-level WAM kernel timing (library HIP events) on the c2 shapes
#   trace/              rocprofv3 --kernel-trace --stats of bench.py (same command as the bench line)
#   pmc_fetch/ pmc_write/  rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs), WAM kernels only
# usage: scripts/profile_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
step() {  # step <seconds> <name> <cmd...>
  local secs=$1 name=$2; shift 2
  echo "=== $name" | tee -a $O/steps.log
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $O/steps.log
  tail -3 $O/$name.log
  return $rc
}
step 150 kbench python3 $R/scripts/kbench.py --iters 20 &&
step 300 trace rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
  python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline off "$@" &&
step 240 pmc_fetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_(plane|ana|adj|dwt|frame|item|noise|cube|subband|acc|trapz|reproj|syn)' --output-format csv -d $O/pmc_fetch -o bench -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-baseline off "$@" &&
step 240 pmc_write rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_(plane|ana|adj|dwt|frame|item|noise|cube|subband|acc|trapz|reproj|syn)' --output-format csv -d $O/pmc_write -o bench -- \
  python3 $R/bench.py --steps 1 --warmup 1 --cpu-baseline off "$@"
