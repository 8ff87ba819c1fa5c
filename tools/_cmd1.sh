set -o pipefail
O=gpurun_out/t2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_errors.py tests/test_configs.py tests/test_table_root.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -20
exit $rc
