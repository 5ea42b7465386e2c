set -euo pipefail
o=gpurun_out/r6k; mkdir -p $o
L=rag-faiss-embedding_amd
# correctness of every arm: the (d) shard at the full 10k batch, 1,000 oracle queries
for v in v5base pm1 pm3 ns6 ka8; do
  FX_INDEX_LIB=$L/libfx_index_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
    "tests/test_configs.py::test_config_shard_full_batch[d-1250000-768-bfloat16-1000]" -m gpu > $o/pytest_$v.log 2>&1
done
ARMS="$L/libfx_index_v5base.so|- $L/libfx_index_pm1.so|- $L/libfx_index_pm3.so|- $L/libfx_index_ns6.so|- $L/libfx_index_ka8.so|-"
bash tools/gpu_multi.sh r6k/d d $ARMS
python tools/show_multi.py gpurun_out/r6k/d > $o/d_summary.txt
BENCH_ARGS="--rows 1250000" bash tools/gpu_multi.sh r6k/shard d $ARMS
python tools/show_multi.py gpurun_out/r6k/shard > $o/shard_summary.txt
echo r6k done
