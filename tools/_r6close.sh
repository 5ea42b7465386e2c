set -euo pipefail
o=gpurun_out/r6close; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
echo r6close done
