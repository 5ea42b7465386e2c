#!/bin/bash
# Round 3: rocprofv3 trace + PMC passes of the config (b) and (e) bench lines
# (so their roofline.traffic is measured, not null).
# usage: tools/r3_prof_be.sh
set -euo pipefail
timeout -k 10 400 tools/profile_scan.sh b --config b --steps 5 --warmup 2
timeout -k 10 600 tools/profile_scan.sh e --config e --steps 3 --warmup 1
echo prof_be done
