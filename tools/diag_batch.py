"""Batch diagnostics: stage-by-stage comparison of one block of a batch with the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402
from tests.helpers import gen, oracle_encode, oracle_stages  # noqa: E402


def main(kind="text", size=4096 * 20 + 9, block=4096, seed=3):
    src = gen(kind, size, seed)
    ctx = salz_amd.Context(0, 1 << 20)
    streams, d = ctx.encode_batch_dump(src, block)
    nb = len(streams)
    bad = []
    for b in range(nb):
        blk = src[b * block:(b + 1) * block]
        rc, ref = oracle_encode(blk)
        if streams[b] != ref:
            bad.append(b)
    print("blocks differing:", bad)
    for b in bad[:2]:
        blk = src[b * block:(b + 1) * block]
        o = oracle_stages(blk)
        n = len(blk) - 8
        p0 = b * block
        # the batch's suffix array: block b's range starts after the earlier blocks' suffixes
        r0 = b * (block - 8)
        sa = d["sa"][r0:r0 + n] - p0
        print(f"block {b}: sa equal {np.array_equal(sa, o['sa'])}")
        for k in ("psv", "nsv"):
            g = d[k][p0:p0 + n].copy()
            g = np.where(g >= 0, g - p0, g)
            i = np.nonzero(g != o[k])[0]
            print(f"  {k}: {len(i)} diffs", [(int(x), int(g[x]), int(o[k][x])) for x in i[:5]])
        for k in ("lp", "ln", "dlen", "doff"):
            g = d[k][p0:p0 + n]
            i = np.nonzero(g != o[k])[0]
            print(f"  {k}: {len(i)} diffs", [(int(x), int(g[x]), int(o[k][x])) for x in i[:5]])
        g = d["cost"][p0:p0 + n + 1]
        i = np.nonzero(g[1:] != o["cost"][1:])[0]
        print(f"  cost: {len(i)} diffs", [(int(x) + 1, int(g[x + 1]), int(o['cost'][x + 1])) for x in i[:5]])




def stream_diff(kind="text", size=4096 * 20 + 9, block=4096, seed=3):
    src = gen(kind, size, seed)
    ctx = salz_amd.Context(0, 1 << 20)
    streams = ctx.encode_batch(src, block)
    for b, s in enumerate(streams):
        rc, ref = oracle_encode(src[b * block:(b + 1) * block])
        if s == ref:
            continue
        i = next(k for k in range(4, min(len(s), len(ref))) if s[k] != ref[k])
        j = 0
        while j < min(len(s), len(ref)) and s[-1 - j] == ref[-1 - j]:
            j += 1
        print(f"block {b}: gpu {len(s)} oracle {len(ref)} first diff at {i}, common suffix {j}")
        print("  gpu   ", s[i - 8:i + 24].hex())
        print("  oracle", ref[i - 8:i + 24].hex())


def tokens(stream):
    """Token list (pos, len) of a SALZ stream (control words MSB-first)."""
    body = stream[4:]
    pos = 0
    bits, avail = 0, 0
    out_pos = 0
    toks = []

    def bit():
        nonlocal bits, avail, pos
        if avail == 0:
            bits = int.from_bytes(body[pos:pos + 8], "little")
            pos += 8
            avail = 64
        avail -= 1
        return (bits >> avail) & 1

    def nbits(k):
        v = 0
        for _ in range(k):
            v = (v << 1) | bit()
        return v

    while pos < len(body) or avail:
        if pos >= len(body) and avail == 0:
            break
        t = bit()
        if t == 0:
            if pos >= len(body):
                break
            pos += 1
            toks.append((out_pos, 1))
            out_pos += 1
            continue
        v = 0
        for i in range(11):
            nib = nbits(4)
            v = (nib & 7) if i == 0 else (((v + 1) << 3) | (nib & 7))
            if nib & 8:
                break
        pos += 1
        q = 0
        while bit() == 0:
            q += 1
        low = nbits(3)
        L = (q << 3 | low) + 3
        toks.append((out_pos, L))
        out_pos += L
    return toks


def token_diff(kind="text", size=4096 * 20 + 9, block=4096, seed=3):
    src = gen(kind, size, seed)
    ctx = salz_amd.Context(0, 1 << 20)
    streams = ctx.encode_batch(src, block)
    for b, s in enumerate(streams):
        rc, ref = oracle_encode(src[b * block:(b + 1) * block])
        if s == ref:
            continue
        tg, to = tokens(s), tokens(ref)
        i = next((k for k in range(min(len(tg), len(to))) if tg[k] != to[k]), min(len(tg), len(to)))
        print(f"block {b}: tokens gpu {len(tg)} oracle {len(to)}; first diff token {i}")
        print("  gpu   ", tg[max(0, i - 3):i + 6])
        print("  oracle", to[max(0, i - 3):i + 6])


def entries(kind="text", size=4096 * 20 + 9, block=4096, seed=3, bad_block=15):
    import ctypes

    src = gen(kind, size, seed)
    ctx = salz_amd.Context(0, 1 << 20)
    streams, d = ctx.encode_batch_dump(src, block)
    K = 1 << salz_amd.lib.salz_gpu_parse_chunk_log(len(src))
    nch = -(-(len(src) - 8) // K)
    ent = np.zeros(nch + 1, np.uint32)
    salz_amd.lib.salz_debug_ws_read.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
    salz_amd.lib.salz_debug_ws_read(ctx.handle, 0, 0, nch + 1, ent.ctypes.data)
    p0 = bad_block * block
    # path from dlen
    path, p = [], p0
    while p < p0 + block - 8:
        path.append(p)
        p += max(1, int(d["dlen"][p]))
    c0, c1 = p0 // K, (p0 + block) // K
    for c in range(c0, c1):
        on = [q for q in path if c * K <= q < (c + 1) * K]
        e = int(ent[c])
        print(f"chunk {c} [{c * K - p0}, {(c + 1) * K - p0}): entry {e - p0 if e != 0xffffffff else None} "
              f"path first {on[0] - p0 if on else None}")


if __name__ == "__main__":
    main(*[int(a) if a.isdigit() else a for a in sys.argv[1:]])
    stream_diff(*[int(a) if a.isdigit() else a for a in sys.argv[1:]])
    entries()
    token_diff(*[int(a) if a.isdigit() else a for a in sys.argv[1:]])


