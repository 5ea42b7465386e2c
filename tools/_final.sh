# Final evidence of the round on ONE box (tools/_final.sh <tag>): the GPU
# suite, smoke, rocprofv3 trace + PMC passes of (d) [(e), (b) with FULL=1],
# the bench lines of (d) (driver default: CPU leg, 1,000-query recall), (e),
# (b), and the block-skew trace of (d).  Stops at the first failure.
set -euo pipefail
tag=$1
o=gpurun_out/$tag; mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
bash tools/profile_scan.sh ${tag}_d
timeout -k 10 600 python -u bench.py > $o/bench_d.json 2> $o/bench_d.err
if [ "${FULL:-1}" = 1 ]; then
  bash tools/profile_scan.sh ${tag}_e --config e --steps 3 --warmup 1
  bash tools/profile_scan.sh ${tag}_b --config b
  timeout -k 10 600 python -u bench.py --config e --steps 5 --warmup 1 > $o/bench_e.json 2> $o/bench_e.err
  timeout -k 10 300 python -u bench.py --config b > $o/bench_b.json 2> $o/bench_b.err
  timeout -k 10 300 python -u tools/block_skew.py --config d > $o/skew_d.json 2> $o/skew_d.err
fi
echo "final $tag done"
