# Round 6 o: the committed HEAD (lazy register-image plans) end to end: smoke and the default bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']), 'img/s', 'fc1 frac', round(r['frac'], 4), 'traffic', r['traffic'], 'mfma_util', r['mfma_util'], {k: round(v['launch_us'], 1) for k, v in d['kernels'].items()}, 'parity', d['parity']['tie_resolved']['pass'])"
