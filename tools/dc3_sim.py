"""CPU model of the GPU DC3 suffix sorter (salz_amd/csrc/gpu/dc3.hip), step for step.

Not the oracle (oracle/salz_oracle.c has its own SA-IS); this checks the decomposition the
kernels use -- sample keys, naming, the dummy suffix, the rank array, the mod-0 list taken
from the sorted sample, the merge comparator -- against a naive suffix sort:

    python tools/dc3_sim.py          # random, periodic and Fibonacci strings
"""
import numpy as np


def naive_sa(t):
    t = list(t)
    return sorted(range(len(t)), key=lambda i: t[i:])


def dc3(t):
    """t: 1-based symbols (numpy int64), no sentinel. Returns the suffix array (numpy)."""
    n = len(t)
    if n == 1:
        return np.zeros(1, np.int64)
    T = np.zeros(n + 4, np.int64)
    T[:n] = t
    dummy = 1 if n % 3 == 1 else 0
    n1 = (n - 1 + 2) // 3 + dummy  # mod-1 positions < n (1, 4, ...) + the dummy at n
    n2 = (n - 2 + 2) // 3 if n >= 2 else 0
    ns = n1 + n2
    # sample positions in R order: R index j < n1 -> 3j + 1, else 3(j - n1) + 2
    j = np.arange(ns)
    pos = np.where(j < n1, 3 * j + 1, 3 * (j - n1) + 2)
    # sort the sample by its triple (stable LSD: the kernels' radix sort)
    b = int(T.max()).bit_length()
    key = (T[pos] << (2 * b)) | (T[pos + 1] << b) | T[pos + 2]
    order = np.argsort(key, kind="stable")
    skey = key[order]
    head = np.ones(ns, bool)
    head[1:] = skey[1:] != skey[:-1]
    names_sorted = np.cumsum(head)  # 1-based names
    D = int(names_sorted[-1])
    R = np.zeros(ns, np.int64)
    R[order] = names_sorted  # R[j] = name of sample j
    if D == ns:
        sa_r = order  # R index of the sample suffix at each sorted position
    else:
        sa_r = dc3(R)
    sa_pos = pos[sa_r]  # sorted sample as text positions (dummy first if any)
    rank = np.zeros(n + 4, np.int64)
    rank[sa_pos] = np.arange(1, ns + 1)
    rank[n:] = 0
    if dummy:
        assert sa_pos[0] == n
        sa_pos = sa_pos[1:]
    # mod-0 suffixes ordered by rank[i + 1]: the mod-1 entries of the sorted sample (dummy
    # included: it stands for i = n - 1), then a stable sort by T[i]
    full_pos = pos[sa_r]
    m1 = full_pos[full_pos % 3 == 1] - 1
    m1 = m1[m1 < n]
    b_list = m1[np.argsort(T[m1], kind="stable")]
    assert len(b_list) == (n + 2) // 3
    # merge with the comparator the merge kernel uses
    def q(p):
        return (T[p], T[p + 1], rank[p + 1], rank[p + 2])

    def b_less_a(bq, aq, a_mod):
        if a_mod == 1:
            return (bq[0], bq[2]) < (aq[0], aq[2])
        return (bq[0], bq[1], bq[3]) < (aq[0], aq[1], aq[3])

    out = []
    ia = ib = 0
    A, B = list(sa_pos), list(b_list)
    while ia < len(A) and ib < len(B):
        if b_less_a(q(B[ib]), q(A[ia]), A[ia] % 3):
            out.append(B[ib])
            ib += 1
        else:
            out.append(A[ia])
            ia += 1
    out += A[ia:] + B[ib:]
    return np.array(out, np.int64)


def fib(n):
    a, b = "b", "a"
    while len(b) < n:
        a, b = b, b + a
    return b[:n]


def main():
    rng = np.random.default_rng(1)
    cases = []
    for n in list(range(1, 40)) + [100, 257, 1000, 1001, 1002]:
        for sigma in (1, 2, 3, 26):
            cases.append(rng.integers(1, sigma + 1, n))
    for n in (1, 2, 3, 4, 5, 10, 100, 1000, 3001):
        cases.append(np.array([1 + (c == "b") for c in fib(n)], np.int64))
        cases.append(np.array([1 + (i % 3) for i in range(n)], np.int64))
    for t in cases:
        got = dc3(t)
        want = naive_sa(t)
        assert list(got) == want, (list(t), list(got), want)
    print(f"dc3 model == naive suffix sort on {len(cases)} strings")


if __name__ == "__main__":
    main()
