set -euo pipefail
o=gpurun_out/r6w; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
bash tools/gpu_multi.sh r6w/d d $L"|-" $L"|FX_CONVOY_EVERY=1 FX_CONVOY_WSTRIDE=4" $L"|FX_CONVOY_EVERY=1 FX_CONVOY_WSTRIDE=8" $L"|FX_CONVOY_EVERY=2 FX_CONVOY_WSTRIDE=2" $L"|FX_CONVOY_EVERY=2 FX_CONVOY_WSTRIDE=4"
python tools/show_multi.py gpurun_out/r6w/d > $o/d_summary.txt
FX_PROFILE_MIN=1 bash tools/profile_scan.sh r6w_e4w1
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=1 FX_CONVOY_WSTRIDE=4 bash tools/profile_scan.sh r6w_e1w4
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=1 FX_CONVOY_WSTRIDE=8 bash tools/profile_scan.sh r6w_e1w8
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=2 FX_CONVOY_WSTRIDE=2 bash tools/profile_scan.sh r6w_e2w2
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=2 FX_CONVOY_WSTRIDE=4 bash tools/profile_scan.sh r6w_e2w4
echo r6w done
