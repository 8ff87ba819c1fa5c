set -o pipefail
O=gpurun_out/b3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 > $O/c3_100M.json 2> $O/c3_100M.err || { tail -20 $O/c3_100M.err; exit 1; }
cat $O/c3_100M.json
echo ok
