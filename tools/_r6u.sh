set -euo pipefail
o=gpurun_out/r6u; mkdir -p $o
L=rag-faiss-embedding_amd/libfx_index.so
bash tools/gpu_multi.sh r6u/d d $L"|-" $L"|FX_CONVOY_EVERY=2" $L"|FX_CONVOY_EVERY=1 FX_CONVOY_SPREAD=1" $L"|FX_CONVOY_EVERY=1 FX_CONVOY_SPREAD=2" $L"|FX_CONVOY_EVERY=1 FX_CONVOY_SPREAD=4" $L"|FX_CONVOY_SPREAD=2"
python tools/show_multi.py gpurun_out/r6u/d > $o/d_summary.txt
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=2 bash tools/profile_scan.sh r6u_e2
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=1 FX_CONVOY_SPREAD=1 bash tools/profile_scan.sh r6u_e1s1
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=1 FX_CONVOY_SPREAD=2 bash tools/profile_scan.sh r6u_e1s2
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=1 FX_CONVOY_SPREAD=4 bash tools/profile_scan.sh r6u_e1s4
FX_PROFILE_MIN=1 FX_CONVOY_SPREAD=2 bash tools/profile_scan.sh r6u_e4s2
echo r6u done
