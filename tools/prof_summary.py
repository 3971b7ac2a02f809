#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: short kernel name, calls, total, average, share.
  python tools/prof_summary.py path/to/run_kernel_stats.csv [--steps K]"""
import csv, re, sys
path = sys.argv[1]
steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 1
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':34s} {'calls':>7s} {'total ms':>10s} {'avg us':>10s} {'share':>7s}")
for r in rows:
    name = r["Name"]
    m = re.search(r"(k_[a-z0-9_]+|__amd_rocclr_[A-Za-z]+)", name)
    short = m.group(1) if m else name[:34]
    if "k_radix" in short and ("ILb1E" in name or "<true>" in name):
        short += "<text>"  # round 0's first pass, keys built from the text
    elif "<unsigned long" in name:
        short += "<u64>"
    elif "MaxOp" in name:
        short += "<max>"
    print(f"{short:34s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:10.3f} "
          f"{float(r['AverageNs'])/1e3:10.2f} {100*float(r['TotalDurationNs'])/tot:6.2f}%")
print(f"{'total':34s} {'':7s} {tot/1e6:10.3f}")
