"""Per-pass kernel times of the parse in a rocprofv3 kernel trace (last encode in the file).

  python tools/parse_passes.py <kernel_trace.csv>
A pass starts at k_parse_chunk; the test kernels before it (k_parse_mark and its range test)
are counted in the pass they precede."""
import collections
import csv
import re
import sys


def kname(full):
    m = re.search(r"(k_\w+)", full)  # (template arguments dropped)
    return m.group(1) if m else full.split("(")[0][:30]


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seeds = [i for i, r in enumerate(rows) if "k_cost_seed" in r["Kernel_Name"]]
    passes, cur = [], collections.OrderedDict()
    for r in rows[seeds[-1]:]:
        n = kname(r["Kernel_Name"])
        if n.startswith("k_emit"):
            break
        if n in ("k_parse_mark", "k_shift_breaks", "k_chunk_reach") and "k_parse_chunk" in cur:
            passes.append(cur)
            cur = collections.OrderedDict()
        if n == "k_parse_chunk" and "k_parse_chunk" in cur:
            passes.append(cur)
            cur = collections.OrderedDict()
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cur[n] = cur.get(n, 0) + d
    passes.append(cur)
    for i, p in enumerate(passes):
        print(i, round(sum(p.values())), {k: round(v) for k, v in p.items() if v > 15})


if __name__ == "__main__":
    main(sys.argv[1])
