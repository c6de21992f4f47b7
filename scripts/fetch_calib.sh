# FETCH_SIZE / WRITE_SIZE per copy width (scripts/ubench_fetch.hip), separate passes
set -o pipefail
cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d /tmp/fc_$c -o run -- $R/scripts/ubench_fetch > /tmp/fc_$c.log 2>&1 || { tail -5 /tmp/fc_$c.log; exit 1; }
  f=$(find /tmp/fc_$c -name "*counter_collection.csv" | head -1)
  python3 -c "
import csv,collections
acc=collections.defaultdict(list)
for r in csv.DictReader(open('$f')):
    acc[r['Kernel_Name'][:40]].append(float(r['Counter_Value']))
for k,v in acc.items(): print('$c', k, ['%.3f GiB' % (x*1024/2**30) for x in v])
"
done
