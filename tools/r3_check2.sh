#!/bin/bash
# Round-3 closing check at HEAD: the whole -m gpu suite, smoke(), and the
# default bench line (no CPU leg).
# usage: tools/r3_check2.sh <tag>
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 \
    || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 \
    || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu > $o/bench_d.json 2> $o/bench_d.err
tail -c 300 $o/bench_d.json
echo check2 done
