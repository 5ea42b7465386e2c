set -euo pipefail
o=gpurun_out/abl1; mkdir -p $o
for d in 0 1 2 3; do
  FX_SCAN_DBG=$d timeout -k 10 120 python -u bench.py --no-cpu --steps 3 --warmup 1 > $o/dbg$d.json 2>$o/dbg$d.err
done
echo ok
