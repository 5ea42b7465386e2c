set -euo pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6b/pytest.log 2>&1
bash tools/lat_trace.sh r6b
timeout -k 10 300 python -u tools/block_skew.py --config d > gpurun_out/r6b/skew_d.json 2> gpurun_out/r6b/skew_d.err
# loop composition of the (d) scan (round-5 ablation build: timing only)
for dbg in 0 8 10 2 4; do
  FX_INDEX_LIB=rag-faiss-embedding_amd/libfx_index_abl.so FX_SCAN_DBG=$dbg timeout -k 10 240 \
    python -u bench.py --no-cpu --latency-calls 0 --steps 5 --warmup 2 > gpurun_out/r6b/abl_d_$dbg.json 2>> gpurun_out/r6b/abl.err
done
echo r6b done
