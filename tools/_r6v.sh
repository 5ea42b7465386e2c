set -euo pipefail
o=gpurun_out/r6v; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
bash tools/gpu_multi.sh r6v/d d $L"|-" $L"|FX_CONVOY_EVERY=1 FX_CONVOY_SLOTS=8" $L"|FX_CONVOY_EVERY=2 FX_CONVOY_SLOTS=8" $L"|FX_CONVOY_SLOTS=8" $L"|FX_CONVOY_SLOTS=4"
python tools/show_multi.py gpurun_out/r6v/d > $o/d_summary.txt
FX_PROFILE_MIN=1 bash tools/profile_scan.sh r6v_e4
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=1 FX_CONVOY_SLOTS=8 bash tools/profile_scan.sh r6v_e1s8
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=2 FX_CONVOY_SLOTS=8 bash tools/profile_scan.sh r6v_e2s8
FX_PROFILE_MIN=1 FX_CONVOY_SLOTS=8 bash tools/profile_scan.sh r6v_e4s8
echo r6v done
