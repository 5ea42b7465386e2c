set -euo pipefail
o=gpurun_out/r6ec; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
bash tools/gpu_multi.sh r6ec/e e $L"|-" $L"|FX_CONVOY=0"
python tools/show_multi.py gpurun_out/r6ec/e > $o/e_summary.txt
FX_PROFILE_MIN=1 bash tools/profile_scan.sh r6ec_e --config e --steps 3 --warmup 1
echo r6ec done
