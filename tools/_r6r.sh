set -euo pipefail
o=gpurun_out/r6r; mkdir -p $o
timeout -k 10 400 python -u tools/_dbg_convoy.py > $o/dbg.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_scan_v5.py -m gpu > $o/pytest_v5.log 2>&1
L=rag-faiss-embedding_amd/libfx_index.so
ARMS="$L|FX_CONVOY=1 $L|FX_CONVOY=0"
bash tools/gpu_multi.sh r6r/d d $ARMS
python tools/show_multi.py gpurun_out/r6r/d > $o/d_summary.txt
BENCH_ARGS="--rows 1250000" bash tools/gpu_multi.sh r6r/shard d $ARMS
python tools/show_multi.py gpurun_out/r6r/shard > $o/shard_summary.txt
FX_PROFILE_MIN=1 FX_CONVOY=1 bash tools/profile_scan.sh r6r_conv1
FX_PROFILE_MIN=1 FX_CONVOY=0 bash tools/profile_scan.sh r6r_conv0
bash tools/gpu_multi.sh r6r/e e $ARMS
python tools/show_multi.py gpurun_out/r6r/e > $o/e_summary.txt
echo r6r done
