set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05af_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05af_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05af_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05af_smoke.log 2>&1 || { tail -20 gpurun_out/r05af_smoke.log; exit 1; }
tail -1 gpurun_out/r05af_smoke.log
rm -rf /tmp/oldtree && cp -r $R /tmp/oldtree && cp $R/build/exp/engine_old.py /tmp/oldtree/wam_amd/engine.py && cp $R/build/exp/wam_2D_old.py /tmp/oldtree/wam_amd/wam_2D.py
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --config c2 --extras off --cpu-baseline off --pmc off 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200 | sed 's/^/new /' | tee -a gpurun_out/r05af_handoff_ab.log || exit 1
  (cd /tmp/oldtree && timeout -k 10 400 python -u bench.py --config c2 --extras off --cpu-baseline off --pmc off 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200 | sed 's/^/old /') | tee -a gpurun_out/r05af_handoff_ab.log || exit 1
done
