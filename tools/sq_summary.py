#!/usr/bin/env python3
"""Per-kernel SQ counters from one rocprofv3 --pmc pass (wave-parked, issue-stalled and active
shares of the wave cycles, VALU and LDS instructions per wave), busiest kernels first.

  rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \\
      SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d DIR -o pmc -- python3 bench.py ...
  python tools/sq_summary.py DIR/pmc_counter_collection.csv [--top N]

WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES (/opt/skills/guides/MI355X_MICROARCH.md,
"rocprofv3 PMC slots"): a kernel parked most of its cycles waits on memory; a high active share
with many VALU instructions per wave is instruction-bound."""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_[a-z0-9_]+|__amd_rocclr_[A-Za-z]+)", r["Kernel_Name"])
        agg[m.group(1) if m else r["Kernel_Name"][:30]][r["Counter_Name"]] += float(r["Counter_Value"])
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["SQ_BUSY_CYCLES"])
    print(f"{'kernel':22s} {'waves':>9s} {'busy cyc':>9s} {'parked%':>7s} {'stall%':>6s} {'active%':>7s} "
          f"{'VALU/wave':>9s} {'LDS/wave':>8s}")
    for name, c in rows[:top]:
        wc = c["SQ_WAVE_CYCLES"] or 1.0
        wv = max(1.0, c["SQ_WAVES"])
        print(f"{name:22s} {c['SQ_WAVES']:9.0f} {c['SQ_BUSY_CYCLES']:9.3g} {100 * c['SQ_WAIT_ANY'] / wc:7.1f} "
              f"{100 * c['SQ_WAIT_INST_ANY'] / wc:6.1f} {100 * c['SQ_ACTIVE_INST_ANY'] / wc:7.1f} "
              f"{c['SQ_INSTS_VALU'] / wv:9.0f} {c['SQ_INSTS_LDS'] / wv:8.0f}")


if __name__ == "__main__":
    main()
