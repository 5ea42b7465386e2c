#!/bin/bash
# Closing check of the tree as committed: the -m gpu suite, smoke(), and the
# default (d) bench line.  Stops at the first failure.
# usage: tools/r4_closecheck.sh <tag>
set -euo pipefail
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
tail -2 $o/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 400 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
tail -c 400 $o/bench_d.json
echo closecheck done
