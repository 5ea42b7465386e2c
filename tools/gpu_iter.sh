#!/bin/bash
# One iteration on the GPU box after a scan change: the scan's key-matrix and
# parity tests (+ the sanitizer ABI run), config (d) bench lines (default and
# corpus-partitioned placement), a stamp run of the -DFX_ABLATION build and a
# kernel-trace profile.  Stops at the first failure.
# usage: tools/gpu_iter.sh <tag>
set -euo pipefail
o=gpurun_out/$1
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_scan_keys.py tests/test_gpu_parity.py tests/test_configs.py tests/test_cert_stress.py tests/test_big_k.py tests/test_q32.py tests/test_native_asan.py > $o/tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > $o/bench_d.json 2> $o/bench_d.err
FX_SCAN_PLACE=1 timeout -k 10 300 python -u bench.py --no-cpu > $o/bench_d_p1.json 2> $o/bench_d_p1.err
FX_INDEX_LIB=rag-faiss-embedding_amd/libfx_index_abl.so FX_SCAN_DBG=64 FX_SCAN_STAMPS=$o/stamps64.bin timeout -k 10 200 python -u bench.py --no-cpu --steps 1 --warmup 1 > $o/st64.json 2> $o/st64.err
python tools/show_stamps.py $o/stamps64.bin > $o/stamps64.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $o/trace.log 2>&1
echo iter done
