set -euo pipefail
o=gpurun_out/r6x; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
bash tools/gpu_multi.sh r6x/e e $L"|-" $L"|FX_CONVOY=0" $L"|FX_CONVOY_EVERY=8"
python tools/show_multi.py gpurun_out/r6x/e > $o/e_summary.txt
FX_PROFILE_MIN=1 bash tools/profile_scan.sh r6x_e4 --config e --steps 3 --warmup 1
FX_PROFILE_MIN=1 FX_CONVOY=0 bash tools/profile_scan.sh r6x_c0 --config e --steps 3 --warmup 1
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=8 bash tools/profile_scan.sh r6x_e8 --config e --steps 3 --warmup 1
echo r6x done
