set -euo pipefail
o=gpurun_out/r6i; mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
bash tools/lat_trace.sh r6i
echo r6i done
