#!/usr/bin/env python3
"""Flag partial vmcnt waits that separate VMEM ops issued under different EXEC masks.

Linear scan of an llvm-objdump disassembly (gfx950 code objects): every VMEM op gets the
current "exec epoch" (bumped by any instruction that writes EXEC); an `s_waitcnt vmcnt(k)`
with k > 0 retires all but the last k ops. A wait that retires an op of one epoch while an
op of another epoch stays outstanding is the shape that returned stale registers under
concurrent GPU load (load_u64_any). Heuristic: branches are not followed.
  python tools/vmcnt_scan.py file.s [...]
"""
import re
import sys

VMEM = re.compile(r"^\s*(global|buffer|flat|scratch)_(load|store|atomic)")
EXECW = re.compile(r"^\s*s_\w+\s+(exec\b|s\[\d+:\d+\],\s*\S+.*saveexec)|saveexec")
WAIT = re.compile(r"s_waitcnt.*vmcnt\((\d+)\)")


def scan(path):
    hits = []
    kern = None
    epoch = 0
    pend = []
    for line in open(path):
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            kern, epoch, pend = m.group(1), 0, []
            continue
        code = line.split("//")[0]
        if VMEM.match(code):
            pend.append(epoch)
        elif "exec" in code and re.match(r"^\s*s_", code) and not code.strip().startswith("s_cbranch"):
            dst = code.split()[1] if len(code.split()) > 1 else ""
            if "saveexec" in code or dst.startswith("exec"):
                epoch += 1
        w = WAIT.search(code)
        if w:
            k = int(w.group(1))
            if k == 0:
                pend = []
            elif len(pend) > k:
                done, out = pend[:-k], pend[-k:]
                if set(out) - set(done) and set(done) - set(out):
                    hits.append((kern, code.strip()))
                pend = out
    return hits


if __name__ == "__main__":
    n = 0
    for p in sys.argv[1:]:
        for kern, c in scan(p):
            print(f"{p}: {kern}: {c}")
            n += 1
    print(f"{n} suspicious partial waits")
