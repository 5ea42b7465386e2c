set -euo pipefail
o=gpurun_out/r6n; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
ARMS="$L|- $L|FX_COMPACT_AT=40 $L|FX_COMPACT_AT=44 $L|FX_PRUNE_RANK=14 $L|FX_PRUNE_RANK=10 $L|FX_UNION_W=32"
bash tools/gpu_multi.sh r6n/d d $ARMS
python tools/show_multi.py gpurun_out/r6n/d > $o/d_summary.txt
BENCH_ARGS="--rows 1250000" bash tools/gpu_multi.sh r6n/shard d $ARMS
python tools/show_multi.py gpurun_out/r6n/shard > $o/shard_summary.txt
echo r6n done
