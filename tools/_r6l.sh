set -euo pipefail
o=gpurun_out/r6l; mkdir -p $o
L=rag-faiss-embedding_amd
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
for v in ns7 ns8; do
  FX_INDEX_LIB=$L/libfx_index_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
    "tests/test_configs.py::test_config_shard_full_batch[d-1250000-768-bfloat16-1000]" -m gpu > $o/pytest_$v.log 2>&1
done
ARMS="$L/libfx_index.so|- $L/libfx_index_ns7.so|- $L/libfx_index_ns8.so|- $L/libfx_index.so|FX_SCAN_V5=0"
bash tools/gpu_multi.sh r6l/d d $ARMS
python tools/show_multi.py gpurun_out/r6l/d > $o/d_summary.txt
BENCH_ARGS="--rows 1250000" bash tools/gpu_multi.sh r6l/shard d $ARMS
python tools/show_multi.py gpurun_out/r6l/shard > $o/shard_summary.txt
echo r6l done
