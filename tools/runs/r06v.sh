# Round 6 v: the committed head once more on a fresh box: GPU suite, smoke, default bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']), 'img/s', 'fc1 frac', round(r['frac'], 4), 'traffic', r['traffic'], 'mfma_util', r['mfma_util'], {k: round(v['launch_us'], 1) for k, v in d['kernels'].items()}, 'parity', d['parity']['tie_resolved']['pass'])"
