"""Split a rocprofv3 kernel trace of one encode into suffix-sort rounds and stages.

  python tools/trace_rounds.py <kernel_trace.csv> [encode index]

An encode starts at the text-sourced radix histogram (round 0); each doubling round ends with
k_commit / k_rank_upper and the next round's k_keys (or, for round 0 whose commit gathers the text
round's keys, with k_commit). Prints per-round kernel time (sum of
dispatch durations) and the wall span, and the per-kernel totals of the later stages."""
import collections
import csv
import re
import sys


def kname(full):
    m = re.search(r"(k_\w+(<[^>]*>)?)", full)
    return m.group(1) if m else full.split("(")[0]


def main(path, which=0):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_radix_hist<1" in r["Kernel_Name"] or "k_radix_hist<3>" in r["Kernel_Name"] or
              "k_radix_hist<true>" in r["Kernel_Name"]]
    if not starts:
        sys.exit("no encode found")
    a = starts[which]
    b = starts[which + 1] if which + 1 < len(starts) else len(rows)
    enc = rows[a:b]
    rounds, cur = [], []
    stage = "sa"
    post = collections.OrderedDict()
    names = [kname(r["Kernel_Name"]) for r in enc]
    for idx, r in enumerate(enc):
        name = names[idx]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if name.startswith("k_ansv_local") or name.startswith("k_phi"):
            stage = "post"
        if stage == "sa":
            cur.append((name, dur, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            nxt = next((x for x in names[idx + 1:] if x != "k_read_scalars"), "")
            # (round 0 before the text round gathers the text keys inside k_commit: no k_keys)
            fused_end = name in ("k_commit", "k_rank_upper") and not nxt.startswith(("k_keys", "k_rank_upper"))
            if name.startswith("k_keys") or fused_end:
                rounds.append(cur)
                cur = []
        else:
            post[name] = post.get(name, 0.0) + dur
    if cur:
        rounds.append(cur)
    total = 0.0
    for k, rd in enumerate(rounds):
        busy = sum(d for _, d, _, _ in rd)
        span = (rd[-1][3] - rd[0][2]) / 1e3
        total += span
        agg = collections.Counter()
        for n, d, _, _ in rd:
            agg[n] += d
        top = ", ".join(f"{n} {d:.0f}" for n, d in agg.most_common(6))
        print(f"round {k}: busy {busy:.0f} us, span {span:.0f} us | {top}")
    print(f"sa span total {total / 1e3:.2f} ms")
    for n, d in sorted(post.items(), key=lambda x: -x[1])[:12]:
        print(f"  post {n}: {d:.0f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
