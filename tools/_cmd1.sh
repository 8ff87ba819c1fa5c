set -o pipefail
O=gpurun_out/t3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
exit $rc
