set -euo pipefail
o=gpurun_out/r6v4c; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_scan_v5.py -m gpu > $o/pytest_v5.log 2>&1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $o/pytest.log 2>&1
L=rag-faiss-embedding_amd/libfx_index.so
BENCH_ARGS="--nq 10000" bash tools/gpu_multi.sh r6v4c/b10k b $L"|-" $L"|FX_CONVOY=0"
python tools/show_multi.py gpurun_out/r6v4c/b10k > $o/b10k_summary.txt
bash tools/gpu_multi.sh r6v4c/b b $L"|-" $L"|FX_CONVOY=0"
python tools/show_multi.py gpurun_out/r6v4c/b > $o/b_summary.txt
FX_PROFILE_MIN=1 bash tools/profile_scan.sh r6v4c_b10k_c1 --config b --nq 10000
FX_PROFILE_MIN=1 FX_CONVOY=0 bash tools/profile_scan.sh r6v4c_b10k_c0 --config b --nq 10000
P="python3 -u tools/latency_probe.py --k 10 --reps 300"
timeout -k 10 120 $P --rows 100000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
echo r6v4c done
