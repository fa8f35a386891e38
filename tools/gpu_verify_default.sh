cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/verify
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_headline_gpu.py -k "stem or gauss or models or headline or golden" -p no:cacheprovider > gpurun_out/verify/pytest.log 2>&1 && tail -1 gpurun_out/verify/pytest.log && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify/smoke.log 2>&1 && tail -2 gpurun_out/verify/smoke.log
