set -euo pipefail
o=gpurun_out/r6g; mkdir -p $o
B="python -u bench.py --no-cpu --latency-calls 0"
for rep in 1 2; do
  for sx in 0 6 9 12; do
    FX_SCAN_SX=$sx timeout -k 10 300 $B --steps 10 --warmup 2 >> $o/sx_d.jsonl 2>> $o/bench.err
  done
  for sx in 0 6 9; do
    FX_SCAN_SX=$sx timeout -k 10 200 $B --rows 1250000 --steps 20 --warmup 3 >> $o/sx_shard.jsonl 2>> $o/bench.err
  done
done
for sx in 0 8 12; do
  FX_SCAN_SX=$sx timeout -k 10 300 $B --config e --steps 4 --warmup 1 >> $o/sx_e.jsonl 2>> $o/bench.err
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="python3 -u tools/latency_probe.py --k 10 --reps 100 --rows 100000 --dim 384 --dtype float32"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  --output-format csv -d $o/pmc_lat -o run -- $P > $o/pmc_lat.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
  --output-format csv -d $o/pmc_lat2 -o run -- $P > $o/pmc_lat2.log 2>&1
echo r6g done
