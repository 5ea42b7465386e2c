#!/bin/bash
# First GPU session for the opt-in scan variants written without hardware:
#   * the 8-wave K-split scan (k_scan_v5, FX_SCAN_V5=1; =2 staggered epilogue),
#   * the corpus-partitioned XCD placement (FX_SCAN_MAP=1),
#   * the split-fp32 scan of fp32 indexes (FX_F32_SPLIT=1),
#   * the small-batch scan k_scan_q32 (FX_SCAN_Q32=1),
#   * the graph-replayed small host search (FX_SEARCH_GRAPH=1).
# Key-matrix and parity tests first, then config (d) / (b) benches back to
# back.  Stops at the first failure (a fault ends the call: no retries).
set -euo pipefail
out=gpurun_out/${1:-exp}
mkdir -p "$out"
FX_TEST_EXPERIMENTAL=1 timeout -k 10 300 python -u -m pytest tests/test_f32_split.py -x -v --timeout 120 --timeout-method thread > "$out/split.log" 2>&1
FX_TEST_EXPERIMENTAL=1 timeout -k 10 300 python -u -m pytest tests/test_q32.py -x -v --timeout 120 --timeout-method thread > "$out/q32.log" 2>&1
for nq in 1 32; do
  timeout -k 10 240 python -u bench.py --config d --nq $nq --no-cpu --steps 20 >> "$out/nq_d_v4.jsonl" 2>> "$out/nq.err"
  FX_SCAN_Q32=1 timeout -k 10 240 python -u bench.py --config d --nq $nq --no-cpu --steps 20 >> "$out/nq_d_q32.jsonl" 2>> "$out/nq.err"
done
timeout -k 10 240 python -u bench.py --config b --no-cpu > "$out/bench_b.json" 2> "$out/bench_b.err"
FX_F32_SPLIT=1 timeout -k 10 240 python -u bench.py --config b --no-cpu > "$out/bench_b_split.json" 2> "$out/bench_b_split.err"
FX_SCAN_V5=1 timeout -k 10 300 python -u -m pytest tests/test_scan_keys.py -x -v --timeout 120 --timeout-method thread > "$out/keys_v5.log" 2>&1
FX_SCAN_V5=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > "$out/parity_v5.log" 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v4.json" 2> "$out/bench_d_v4.err"
FX_SCAN_V5=1 timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v5.json" 2> "$out/bench_d_v5.err"
FX_SCAN_V5=2 timeout -k 10 300 python -u -m pytest tests/test_scan_keys.py -x -v --timeout 120 --timeout-method thread > "$out/keys_v5s.log" 2>&1
FX_SCAN_V5=2 timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v5s.json" 2> "$out/bench_d_v5s.err"
# corpus-partitioned XCD placement (FX_SCAN_MAP=1) with each kernel
FX_SCAN_MAP=1 timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v4_map.json" 2> "$out/bench_d_v4_map.err"
FX_SCAN_MAP=1 FX_SCAN_V5=1 timeout -k 10 300 python -u bench.py --no-cpu > "$out/bench_d_v5_map.json" 2> "$out/bench_d_v5_map.err"
FX_TEST_EXPERIMENTAL=1 timeout -k 10 300 python -u -m pytest tests/test_search_graph.py -x -v --timeout 120 --timeout-method thread > "$out/graph.log" 2>&1
# single-query latency, the reference's call form (config b / d shapes)
for envs in "" "FX_SCAN_Q32=1" "FX_SCAN_Q32=1 FX_SEARCH_GRAPH=1" "FX_SCAN_Q32=1 FX_SEARCH_GRAPH=1 FX_F32_SPLIT=1"; do
  (
    if [ -n "$envs" ]; then export $envs; fi
    export FX_SEARCH_GRAPH_VERBOSE=1
    timeout -k 10 200 python -u tools/latency_probe.py >> "$out/latency_b.jsonl" 2>> "$out/latency.err"
    timeout -k 10 300 python -u tools/latency_probe.py --rows 10000000 --dim 768 --dtype bfloat16 \
      >> "$out/latency_d.jsonl" 2>> "$out/latency.err"
  )
done
echo done
