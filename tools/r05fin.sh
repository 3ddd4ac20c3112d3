set -u
O=gpurun_out/${OUTD:-r05fin}; mkdir -p $O; export TMPDIR=/tmp
(while sleep 50; do date >> $O/heartbeat.txt; done) & HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 300 python bench.py --model ultranet --batch 256 > $O/ultra.log 2>&1 || { echo "ultranet bench failed"; tail -20 $O/ultra.log; exit 1; }
grep '^{' $O/ultra.log > $O/ultra.json; cut -c1-300 $O/ultra.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_ultra -o ultra -- python bench.py --model ultranet --batch 256 --steps 5 --warmup 2 --no-cpu-baseline > $O/rp_ultra.log 2>&1 || { echo "ultranet rocprof failed"; tail -20 $O/rp_ultra.log; exit 1; }
timeout -k 10 900 python bench.py --model vit_large_patch16_384 --batch 128 > $O/vitl.log 2>&1 || { echo "vitl bench failed"; tail -20 $O/vitl.log; exit 1; }
grep '^{' $O/vitl.log > $O/vitl.json; cut -c1-300 $O/vitl.json
