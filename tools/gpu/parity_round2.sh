set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_restated.py tests/test_gpu_hierarchical.py -v -s --timeout 180 --timeout-method thread > gpurun_out/new_tests.log 2>&1
rc=$?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread --deselect tests/test_gpu_restated.py --deselect tests/test_gpu_hierarchical.py > gpurun_out/gpu_rest.log 2>&1
echo "rc new=$rc rest=$?"
