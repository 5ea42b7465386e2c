set -euo pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6b/pytest.log 2>&1
bash tools/lat_trace.sh r6b
