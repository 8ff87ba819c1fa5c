set -o pipefail
O=gpurun_out/b8; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "snappy or v2 or multipart or c5" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
DK_SNAPPY_MODE=page timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "snappy or v2 or multipart or c5" > $O/pytest_page.log 2>&1 || { tail -30 $O/pytest_page.log; exit 1; }
tail -1 $O/pytest_page.log
for m in page; do
DK_SNAPPY_MODE=$m timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --workdir /tmp/c3w > $O/c3_$m.json 2> $O/c3_$m.err || { tail -20 $O/c3_$m.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c3_$m.json').read().strip().splitlines()[-1]); print('$m', d['ms_per_step'], d['kernels_us'])"
done
