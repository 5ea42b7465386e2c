set -o pipefail
mkdir -p gpurun_out/r6s
timeout -k 10 400 python -u tools/_dbg_convoy.py > gpurun_out/r6s/dbg.log 2>&1
