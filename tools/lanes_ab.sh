cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out; mkdir -p $O
for r in 1 2; do
for v in "" "--lanes 2" "--lanes 2 --chunk-mib 1024" "--chunk-mib 1024"; do
  timeout -k 10 200 python3 -u bench.py --no-extras $v > $O/ln.json 2> $O/ln.err || { echo "$v failed"; tail -5 $O/ln.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/ln.json'))
print('[$v]', 'value=%.4g' % d['value'], 'ms=%.3f' % d['ms_per_step'])"
done; done
