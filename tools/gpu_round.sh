#!/bin/bash
# One GPU-box session: parity tests, the default bench line, a placement trace
# of the scan, and the rocprofv3 evidence.  Every GPU step has its own time
# limit and the steps stop at the first failure.
set -euo pipefail
out=gpurun_out/${1:-r1}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
timeout -k 10 300 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 python -u bench.py --config b > "$out/bench_b.json" 2> "$out/bench_b.err"
timeout -k 10 400 python -u bench.py --config e --steps 5 > "$out/bench_e.json" 2> "$out/bench_e.err"
timeout -k 10 400 python -u tools/bench_e2e.py > "$out/bench_c.json" 2> "$out/bench_c.err"
FX_SCAN_TRACE="$out/scan_trace.bin" timeout -k 10 200 python -u bench.py --no-cpu --steps 1 --warmup 1 > "$out/trace_bench.json" 2>&1
python tools/analyze_trace.py "$out/scan_trace.bin" > "$out/trace.txt" 2>&1 || true
echo done
