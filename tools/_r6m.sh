set -euo pipefail
o=gpurun_out/r6m; mkdir -p $o
L=rag-faiss-embedding_amd
for v in e6 e540; do
  FX_INDEX_LIB=$L/libfx_index_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread \
    "tests/test_configs.py::test_config_shard_full_batch[e-12500000-384-float16-512]" -m gpu > $o/pytest_$v.log 2>&1
done
ARMS="$L/libfx_index_eb.so|- $L/libfx_index_e6.so|- $L/libfx_index_e540.so|-"
bash tools/gpu_multi.sh r6m/e e $ARMS
python tools/show_multi.py gpurun_out/r6m/e > $o/e_summary.txt
echo r6m done
