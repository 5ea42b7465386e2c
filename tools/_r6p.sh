set -o pipefail
mkdir -p gpurun_out/r6p
timeout -k 10 300 python -u tools/_dbg_small.py > gpurun_out/r6p/dbg.log 2>&1
