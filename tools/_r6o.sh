set -euo pipefail
o=gpurun_out/r6q; mkdir -p $o
timeout -k 10 300 python -u tools/_dbg_small.py > $o/dbg.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_scan_v5.py -m gpu > $o/pytest_v5.log 2>&1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
echo r6q done
