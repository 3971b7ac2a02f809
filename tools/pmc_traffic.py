#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes of the same bench command.

  python tools/pmc_traffic.py FETCH_DIR/pmc_counter_collection.csv WRITE_DIR/pmc_counter_collection.csv \
      [--kernel k_radix_scatter] [--json bench_traffic.json] [--summary out.txt]

Correction (/opt/skills/guides/MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads, so
traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 per dispatch.
Calibrated for the other access widths in round 5 (profiles/r05i_pmc_calibration.txt,
tools/gather_bench calib): every L2 -> fabric read request is a 128-B line whatever the width
(TCC_EA0_RDREQ_128B_sum = TCC_EA0_RDREQ_sum for random 4- and 8-byte reads too) and FETCH_SIZE
tallies 64 B per request, so the x2 holds for every read; a random 4-byte read costs 1.03 lines,
an unaligned 8-byte one 1.08. Infinity Cache hits are counted as traffic: a kernel whose random
side fits the 256 MiB cache can show more than the ~6.3 TB/s HBM delivers (a gather over a
64 MiB table: 7.0 TB/s). WRITE_SIZE is exact for streaming stores; a random 4- or 16-byte store
counts one 32-B sector.

Algorithmic bytes of k_radix_scatter: 24 B per element (read 8 B key + 4 B value, write
8 B key + 4 B value; passes followed by another key pass also write the next digit byte, 25 B,
which bench.py counts exactly); elements per dispatch = Grid_Size / 256 * 4096 (4096-element
tiles, the last tile may be partial, so this is an upper bound within one tile).
"""
import argparse
import collections
import csv
import json
import re


def load(path):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_[a-z0-9_]+|__amd_rocclr_[A-Za-z]+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        if "unsigned long" in r["Kernel_Name"] and name.startswith("k_scan"):
            name += "<u64>"
        if name.startswith("k_radix") and ("ILb1E" in r["Kernel_Name"] or "<true>" in r["Kernel_Name"]):
            name += "<text>"  # round 0's first pass (keys from the text): not the priced kernel
        per[name].append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), int(r["Grid_Size"])))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--kernel", default="k_radix_scatter")
    ap.add_argument("--json")
    ap.add_argument("--summary")
    ap.add_argument("--workload", default="bench.py default (100,000,000-byte text block, 1 step)")
    ap.add_argument("--kind", default="text")
    ap.add_argument("--size", type=int, default=100_000_000)
    a = ap.parse_args()
    F, W = load(a.fetch), load(a.write)
    lines = [f"{'kernel':28s} {'launches':>8s} {'fetch MB':>10s} {'write MB':>10s} {'traffic MB/launch':>18s}"]
    for k in sorted(F, key=lambda k: -sum(v for _, v, _ in F[k])):
        f = sum(v for _, v, _ in F[k]) * 1024 * 2
        w = sum(v for _, v, _ in W.get(k, [])) * 1024
        c = len(F[k])
        lines.append(f"{k:28s} {c:8d} {f / 1e6:10.1f} {w / 1e6:10.1f} {(f + w) / c / 1e6:18.2f}")
    text = "\n".join(lines)
    print(text)
    if a.summary:
        open(a.summary, "w").write(text + "\n")
    fk, wk = F[a.kernel], W[a.kernel]
    launches = len(fk)
    fetch = sum(v for _, v, _ in fk) * 1024 * 2 / launches
    write = sum(v for _, v, _ in wk) * 1024 / len(wk)
    elems = sum(g // 256 * 4096 for _, _, g in fk) / launches
    out = {
        "kernel": a.kernel,
        "workload": a.workload,
        "kind": a.kind,
        "size": a.size,
        "launches": launches,
        "fetch_bytes_per_launch": round(fetch),
        "write_bytes_per_launch": round(write),
        "traffic_per_launch": round(fetch + write),
        "alg_bytes_per_launch_upper": round(24 * elems),
        "traffic_over_alg": round((fetch + write) / (24 * elems), 3),
        "correction": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM section)",
    }
    print(json.dumps(out))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
