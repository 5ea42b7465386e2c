set -euo pipefail
o=gpurun_out/r6h; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 -u tools/latency_probe.py --k 10 --reps 300"
for rep in 1 2; do
  timeout -k 10 120 $P --rows 100000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
  timeout -k 10 120 $P --rows 1000000 --dim 384 --dtype float32 >> $o/latency.jsonl 2>> $o/latency.err
done
P="python3 -u tools/latency_probe.py --k 10 --reps 100 --rows 100000 --dim 384 --dtype float32"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  --output-format csv -d $o/pmc_lat -o run -- $P > $o/pmc_lat.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
  --output-format csv -d $o/pmc_lat2 -o run -- $P > $o/pmc_lat2.log 2>&1
echo r6h done
