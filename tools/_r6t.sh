set -euo pipefail
o=gpurun_out/r6t; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_scan_v5.py -m gpu > $o/pytest_v5.log 2>&1
L=rag-faiss-embedding_amd/libfx_index.so
bash tools/gpu_multi.sh r6t/d d $L"|-" $L"|FX_CONVOY_EVERY=1" $L"|FX_CONVOY_LAG=2" $L"|FX_CONVOY_EVERY=1 FX_CONVOY_LAG=4" $L"|FX_CONVOY_EVERY=8"
python tools/show_multi.py gpurun_out/r6t/d > $o/d_summary.txt
BENCH_ARGS="--rows 1250000" bash tools/gpu_multi.sh r6t/shard d $L"|-" $L"|FX_CONVOY_EVERY=1" $L"|FX_CONVOY_LAG=2"
python tools/show_multi.py gpurun_out/r6t/shard > $o/shard_summary.txt
FX_PROFILE_MIN=1 bash tools/profile_scan.sh r6t_e4l0
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=1 bash tools/profile_scan.sh r6t_e1l0
FX_PROFILE_MIN=1 FX_CONVOY_LAG=2 bash tools/profile_scan.sh r6t_e4l2
FX_PROFILE_MIN=1 FX_CONVOY_EVERY=1 FX_CONVOY_LAG=4 bash tools/profile_scan.sh r6t_e1l4
echo r6t done
