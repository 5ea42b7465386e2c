set -euo pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 600 python -u -m pytest tests/test_scan_options.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6a/pytest.log 2>&1
bash tools/lat_trace.sh r6a
