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
    """EXEC masks are modelled as a stack of regions: `s_and_saveexec` opens a region, `s_xor`,
    `s_or_saveexec` / `s_andn2_saveexec` on EXEC switch to the sibling (else) region, `s_or_b64 exec, exec, s`
    and `s_mov_b64 exec, s` join back to the enclosing one, and other EXEC writes (loop masks,
    atomic optimisations) start a new region in place. Each VMEM op records its region. The block
    after an unconditional `s_branch` starts with no outstanding ops (it is entered by jumps)."""
    hits = []
    kern = None
    stack, nxt, pend = [0], 1, []
    after_jump = False
    for line in open(path):
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            kern, stack, nxt, pend = m.group(1), [0], 1, []
            after_jump = False
            continue
        code = line.split("//")[0].strip()
        if not code:
            continue
        op = code.split()[0]
        args = code[len(op):].replace(" ", "")
        if after_jump:
            # the block after an unconditional jump is entered only by branches, whose
            # outstanding ops this linear scan does not know: start it with none
            pend, after_jump = [], False
        if op == "s_branch":
            after_jump = True
        if VMEM.match(code):
            pend.append(stack[-1])
        elif op.startswith("s_") and not op.startswith("s_cbranch") and (
                "saveexec" in op or args.startswith("exec,") or args.startswith("exec")):
            if op == "s_and_saveexec_b64":
                stack.append(nxt)
            elif op in ("s_andn2_saveexec_b64", "s_or_saveexec_b64") or (
                    op == "s_xor_b64" and args.startswith("exec,exec")):
                stack[-1] = nxt  # else-entry of an if/else: a sibling region
            elif (op == "s_or_b64" and args.startswith("exec,exec,")) or (
                    op == "s_mov_b64" and args.startswith("exec,")):
                if len(stack) > 1:
                    stack.pop()
                nxt -= 1  # no new region opened
            else:
                stack[-1] = nxt
            nxt += 1
        w = WAIT.search(code)
        if w:
            k = int(w.group(1))
            if k == 0:
                pend = []
            elif len(pend) > k:
                done, out = pend[:-k], pend[-k:]
                if set(out) - set(done) and set(done) - set(out):
                    hits.append((kern, code))
                pend = out
    return hits


if __name__ == "__main__":
    n = 0
    for p in sys.argv[1:]:
        for kern, c in scan(p):
            print(f"{p}: {kern}: {c}")
            n += 1
    print(f"{n} suspicious partial waits")
