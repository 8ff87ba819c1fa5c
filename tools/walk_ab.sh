set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/walk_ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_snappy_modes.py tests/test_gpu_parity.py tests/test_errors.py tests/test_plain_strings.py > gpurun_out/walk_ab/pytest.log 2>&1 || { tail -30 gpurun_out/walk_ab/pytest.log; exit 1; }
tail -2 gpurun_out/walk_ab/pytest.log
timeout -k 10 500 bash tools/snap_variants.sh walk_ab/var13 default variants/step96.so variants/budget16.so default variants/step96.so variants/budget16.so > gpurun_out/walk_ab/var.log 2>&1
cat gpurun_out/walk_ab/var.log
