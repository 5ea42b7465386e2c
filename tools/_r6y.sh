set -euo pipefail
o=gpurun_out/r6y; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_scan_v5.py -m gpu > $o/pytest_v5.log 2>&1
L=rag-faiss-embedding_amd/libfx_index.so
bash tools/gpu_multi.sh r6y/d d $L"|-" $L"|FX_CONVOY_STAGGER=1" $L"|FX_CONVOY_STAGGER=1 FX_CONVOY_EVERY=8" $L"|FX_CONVOY_STAGGER=1 FX_CONVOY_EVERY=2"
python tools/show_multi.py gpurun_out/r6y/d > $o/d_summary.txt
FX_PROFILE_MIN=1 bash tools/profile_scan.sh r6y_s0e4
FX_PROFILE_MIN=1 FX_CONVOY_STAGGER=1 bash tools/profile_scan.sh r6y_s1e4
FX_PROFILE_MIN=1 FX_CONVOY_STAGGER=1 FX_CONVOY_EVERY=8 bash tools/profile_scan.sh r6y_s1e8
FX_PROFILE_MIN=1 FX_CONVOY_STAGGER=1 FX_CONVOY_EVERY=2 bash tools/profile_scan.sh r6y_s1e2
BENCH_ARGS="--rows 1250000" bash tools/gpu_multi.sh r6y/shard d $L"|-" $L"|FX_CONVOY_STAGGER=1"
python tools/show_multi.py gpurun_out/r6y/shard > $o/shard_summary.txt
echo r6y done
