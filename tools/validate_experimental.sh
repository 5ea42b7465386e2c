#!/bin/bash
# First GPU sessions for the opt-in variants written without hardware
# (DESIGN.md 3.3), one stage per gpurun call, lowest risk first:
#   low  : split-fp32 scan (FX_F32_SPLIT=1, k_scan_v4<F32S>), corpus-partitioned
#          placement (FX_SCAN_MAP=1), graph-replayed host search (FX_SEARCH_GRAPH=1)
#   q32  : small-batch scan k_scan_q32 (FX_SCAN_Q32=1) + single-query latency
#   v5   : 8-wave K-split scan k_scan_v5 (FX_SCAN_V5=1; =2 staggered epilogue)
# Tests before benches; the script stops at the first failure (a fault ends
# the call: no retries).
# usage: tools/validate_experimental.sh <tag> low|q32|v5
set -euo pipefail
out=gpurun_out/${1:-exp}
stage=${2:-low}
mkdir -p "$out"
T="timeout -k 10"
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"

if [ "$stage" = low ]; then
  FX_TEST_EXPERIMENTAL=1 $T 300 $PYT tests/test_f32_split.py > "$out/split.log" 2>&1
  $T 240 python -u bench.py --config b --no-cpu > "$out/bench_b.json" 2> "$out/bench_b.err"
  FX_F32_SPLIT=1 $T 240 python -u bench.py --config b --no-cpu > "$out/bench_b_split.json" 2> "$out/bench_b_split.err"
  FX_SCAN_MAP=1 $T 300 $PYT tests/test_gpu_parity.py -k large_synth > "$out/parity_map.log" 2>&1  # >= 32 tiles: MAP active
  $T 300 python -u bench.py --no-cpu > "$out/bench_d_v4.json" 2> "$out/bench_d_v4.err"
  FX_SCAN_MAP=1 $T 300 python -u bench.py --no-cpu > "$out/bench_d_v4_map.json" 2> "$out/bench_d_v4_map.err"
  FX_TEST_EXPERIMENTAL=1 $T 300 $PYT "tests/test_search_graph.py::test_graph_replay_matches_oracle[0]" \
    tests/test_search_graph.py::test_graph_store_single_queries > "$out/graph.log" 2>&1  # [1] (q32) in stage q32
  FX_SEARCH_GRAPH=1 FX_SEARCH_GRAPH_VERBOSE=1 $T 200 python -u tools/latency_probe.py >> "$out/latency_b.jsonl" 2>> "$out/latency.err"
  $T 200 python -u tools/latency_probe.py >> "$out/latency_b.jsonl" 2>> "$out/latency.err"
fi

if [ "$stage" = q32 ]; then
  FX_TEST_EXPERIMENTAL=1 $T 300 $PYT tests/test_q32.py > "$out/q32.log" 2>&1
  FX_TEST_EXPERIMENTAL=1 $T 300 $PYT tests/test_search_graph.py > "$out/graph_q32.log" 2>&1
  for nq in 1 32; do
    $T 240 python -u bench.py --config d --nq $nq --no-cpu --steps 20 >> "$out/nq_d_v4.jsonl" 2>> "$out/nq.err"
    FX_SCAN_Q32=1 $T 240 python -u bench.py --config d --nq $nq --no-cpu --steps 20 >> "$out/nq_d_q32.jsonl" 2>> "$out/nq.err"
  done
  for envs in "FX_SCAN_Q32=1" "FX_SCAN_Q32=1 FX_SEARCH_GRAPH=1" "FX_SCAN_Q32=1 FX_SEARCH_GRAPH=1 FX_F32_SPLIT=1"; do
    (
      export $envs
      $T 200 python -u tools/latency_probe.py >> "$out/latency_b.jsonl" 2>> "$out/latency.err"
      $T 300 python -u tools/latency_probe.py --rows 10000000 --dim 768 --dtype bfloat16 \
        >> "$out/latency_d.jsonl" 2>> "$out/latency.err"
    )
  done
fi

if [ "$stage" = v5 ]; then
  FX_SCAN_V5=1 $T 300 $PYT tests/test_scan_keys.py > "$out/keys_v5.log" 2>&1
  FX_SCAN_V5=1 $T 300 $PYT tests/test_gpu_parity.py > "$out/parity_v5.log" 2>&1
  FX_SCAN_V5=1 $T 300 python -u bench.py --no-cpu > "$out/bench_d_v5.json" 2> "$out/bench_d_v5.err"
  FX_SCAN_V5=1 FX_SCAN_MAP=1 $T 300 python -u bench.py --no-cpu > "$out/bench_d_v5_map.json" 2> "$out/bench_d_v5_map.err"
  FX_SCAN_V5=2 $T 300 $PYT tests/test_scan_keys.py > "$out/keys_v5s.log" 2>&1
  FX_SCAN_V5=2 $T 300 python -u bench.py --no-cpu > "$out/bench_d_v5s.json" 2> "$out/bench_d_v5s.err"
  FX_SCAN_V5=2 FX_SCAN_MAP=1 $T 300 python -u bench.py --no-cpu > "$out/bench_d_v5s_map.json" 2> "$out/bench_d_v5s_map.err"
  # split fp32 on the 8-wave scan (quarter of each plane per wave half)
  FX_SCAN_V5=1 FX_TEST_EXPERIMENTAL=1 $T 300 $PYT tests/test_f32_split.py > "$out/split_v5.log" 2>&1
  FX_SCAN_V5=1 FX_F32_SPLIT=1 $T 240 python -u bench.py --config b --no-cpu > "$out/bench_b_split_v5.json" 2> "$out/bench_b_split_v5.err"
fi
echo "stage $stage done"
