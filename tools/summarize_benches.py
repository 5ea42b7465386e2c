#!/usr/bin/env python3
"""One table from a directory of bench.py / bench_e2e.py JSON outputs
(*.json, *.jsonl), e.g. what tools/validate_experimental.sh or
tools/sweep_nq.sh left under gpurun_out/<tag>/.

usage: tools/summarize_benches.py gpurun_out/exp [more dirs...]
"""
import json
import sys
from pathlib import Path


def rows(path: Path):
    for line in path.read_text().splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                yield json.loads(line)
            except json.JSONDecodeError:
                continue


def main():
    hdr = f"{'file':34s} {'cfg':3s} {'nq':>6s} {'value':>12s} {'scan ms':>9s} {'bound':5s} {'frac':>6s} {'recall':>6s} kernel"
    print(hdr)
    print("-" * len(hdr))
    for d in sys.argv[1:]:
        for f in sorted(Path(d).glob("*.json*")):
            for j in rows(f):
                cfg = j.get("config", {})
                roof = j.get("roofline", {})
                if "build_chunks_per_s" in j:  # bench_e2e.py
                    print(f"{f.name:34s} {'c':3s} {'':>6s} {j['build_chunks_per_s']:>12.1f} {'':>9s} {'':5s} "
                          f"{'':>6s} {j.get('recall_at_10', ''):>6} e2e: {j.get('query_per_s')} q/s")
                    continue
                print(f"{f.name:34s} {str(cfg.get('baseline_config', '')):3s} {cfg.get('nq', ''):>6} "
                      f"{j.get('value', 0):>12.1f} {roof.get('kernel_ms_avg', 0):>9.3f} {roof.get('bound', ''):5s} "
                      f"{roof.get('frac', 0):>6.3f} {str(j.get('recall_at_10', '')):>6s} {roof.get('kernel', '')[:40]}")


if __name__ == "__main__":
    main()
