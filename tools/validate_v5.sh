#!/bin/bash
# First GPU session for the 8-wave scan (k_scan_v5, FX_SCAN_V5=1): key-matrix
# and parity tests with v5 selected, then config (d) with v4 and v5 back to
# back, each also with the corpus-partitioned placement.  Stops at the first failure (a fault ends the call: no retries).
set -euo pipefail
out=gpurun_out/${1:-v5}
mkdir -p "$out"
FX_SCAN_V5=1 timeout -k 10 300 python -u -m pytest tests/test_scan_keys.py -x -v --timeout 120 --timeout-method thread > "$out/keys_v5.log" 2>&1
FX_SCAN_V5=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > "$out/parity_v5.log" 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v4.json" 2> "$out/bench_d_v4.err"
FX_SCAN_V5=1 timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v5.json" 2> "$out/bench_d_v5.err"
# corpus-partitioned XCD placement (FX_SCAN_MAP=1) with each kernel
FX_SCAN_MAP=1 timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v4_map.json" 2> "$out/bench_d_v4_map.err"
FX_SCAN_MAP=1 FX_SCAN_V5=1 timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v5_map.json" 2> "$out/bench_d_v5_map.err"
echo done
