set -euo pipefail
o=gpurun_out/r6sx; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
bash tools/gpu_multi.sh r6sx/e e $L"|-" $L"|FX_SCAN_SX=6" $L"|FX_SCAN_SX=8"
python tools/show_multi.py gpurun_out/r6sx/e > $o/e_summary.txt
FX_PROFILE_MIN=1 FX_SCAN_SX=8 bash tools/profile_scan.sh r6sx_e_sx8 --config e --steps 3 --warmup 1
FX_PROFILE_MIN=1 bash tools/profile_scan.sh r6sx_e_sx4 --config e --steps 3 --warmup 1
bash tools/gpu_multi.sh r6sx/d d $L"|-" $L"|FX_SCAN_SX=4" $L"|FX_SCAN_SX=6"
python tools/show_multi.py gpurun_out/r6sx/d > $o/d_summary.txt
echo r6sx done
