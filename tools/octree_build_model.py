# Numpy model of the device octree build (octree_gpu.hip), checked against the host builder.
# Design aid only (slow pure-Python loops; small inputs): python3 tools/octree_build_model.py
import sys, numpy as np
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))
import iterativeclosestpoint_amd as icp

def lcp_levels(a, b, maxd):
    x = np.bitwise_xor(a, b).astype(np.uint64)
    out = np.full(len(x), maxd, np.int64)
    nz = x != 0
    # highest set bit position
    hb = np.floor(np.log2(x[nz].astype(np.float64))).astype(np.int64)
    # float log2 can be off for big ints; fix
    xs = x[nz]
    hb = np.array([int(v).bit_length() - 1 for v in xs], np.int64)
    # level l (1-based) occupies bits [3*(maxd-l), 3*(maxd-l)+3)
    # first differing level = maxd - hb//3 ; common = that - 1
    out[nz] = maxd - hb // 3 - 1
    return out

def proto(xyz, m, maxd):
    M = len(xyz)
    lo = xyz.min(0) - 0.001; hi = xyz.max(0) + 0.001
    key = np.zeros(M, np.uint64)
    L = np.tile(lo, (M, 1)); H = np.tile(hi, (M, 1))
    for l in range(1, maxd + 1):
        mid = (L + H) / 2
        b = xyz > mid
        o = b[:, 0] * 1 + b[:, 1] * 2 + b[:, 2] * 4
        key |= o.astype(np.uint64) << np.uint64(3 * (maxd - l))
        L = np.where(b, mid, L); H = np.where(b, H, mid)
    order = np.argsort(key, kind="stable")
    K = key[order]
    m = max(m, 0)
    if M > m:
        Lw = lcp_levels(K[: M - m], K[m:], maxd)  # j in [0, M-1-m]
        D = np.empty(M, np.int64)
        for i in range(M):
            a, bb = max(0, i - m), min(i, M - 1 - m)
            D[i] = min(maxd, 1 + Lw[a:bb + 1].max())
    else:
        D = np.zeros(M, np.int64)
    shift = (3 * (maxd - D)).astype(np.uint64)
    TK = (K >> shift) << shift
    TKo = np.empty(M, np.uint64); TKo[order] = TK
    Do = np.empty(M, np.int64); Do[order] = D
    idx2 = np.argsort(TKo, kind="stable")
    TKs = TKo[idx2]; D2 = Do[idx2]
    c = np.empty(M, np.int64); c[0] = -1
    if M > 1:
        c[1:] = np.minimum(np.minimum(lcp_levels(TKs[1:], TKs[:-1], maxd), D2[1:]), D2[:-1])
    n = D2 - c
    base = np.concatenate([[0], np.cumsum(n)[:-1]])
    Nn = int(n.sum())
    ns = np.empty(Nn, np.int64); nd = np.empty(Nn, np.int64)
    for j in range(M):
        for d in range(c[j] + 1, D2[j] + 1):
            r = base[j] + d - c[j] - 1
            ns[r] = j; nd[r] = d
    leafflag = n > 0
    starts = np.nonzero(leafflag)[0]
    nxt = np.concatenate([starts[1:], [M]])
    leafcount = np.zeros(M, np.int64); leafcount[starts] = nxt - starts
    lvorder = np.argsort(nd, kind="stable")
    off = np.concatenate([[0], np.cumsum(np.bincount(nd, minlength=maxd + 2))])
    lpos = np.empty(Nn, np.int64); lpos[lvorder] = np.arange(Nn) - off[nd[lvorder]]
    parent = np.full(Nn, -1, np.int64)
    for r in range(1, Nn):
        d = nd[r]
        lst = lvorder[off[d - 1]:off[d]]
        k = np.searchsorted(lst, r) - 1
        parent[r] = lst[k]
    nch = np.zeros(Nn, np.int64); mask = np.zeros(Nn, np.int64)
    def octant(r):
        return int((int(TKs[ns[r]]) >> (3 * (maxd - nd[r]))) & 7)
    for r in range(1, Nn):
        nch[parent[r]] += 1; mask[parent[r]] |= 1 << octant(r)
    fc = 1 + np.concatenate([[0], np.cumsum(nch)[:-1]])
    ids = np.zeros(Nn, np.int64)
    for r in range(1, Nn):
        p = parent[r]
        ids[r] = fc[p] + lpos[r] - lpos[p + 1]
    box = np.zeros((Nn, 6)); first = np.zeros(Nn, np.int64); meta = np.zeros(Nn, np.uint64); dep = np.zeros(Nn, np.int64)
    for r in range(Nn):
        j, d = ns[r], nd[r]
        l0 = lo.copy(); h0 = hi.copy()
        for l in range(1, d + 1):
            o = (int(TKs[j]) >> (3 * (maxd - l))) & 7
            for a in range(3):
                mid = (l0[a] + h0[a]) / 2
                if (o >> a) & 1: l0[a] = mid
                else: h0[a] = mid
        i = ids[r]
        box[i, :3] = l0; box[i, 3:] = h0
        if d == D2[j]:
            first[i] = j; meta[i] = 0x80000000 | leafcount[j]
        else:
            first[i] = fc[r]; meta[i] = mask[r]
        dep[i] = d
    return dict(box=box, first=first, meta=meta, depth=dep, orig=idx2, pts=xyz[idx2])

def check(xyz, m, maxd):
    h = icp.octree_build(xyz, m, maxd)
    p = proto(xyz, m, maxd)
    ok = True
    for k in ("box", "first", "meta", "depth", "orig", "pts"):
        a, b = np.asarray(h[k]), np.asarray(p[k])
        if a.shape != b.shape or not np.array_equal(a.astype(b.dtype) if k != "box" and k != "pts" else a, b):
            print("MISMATCH", k, a.shape, b.shape); ok = False
    print("ok" if ok else "FAIL", len(xyz), m, maxd, len(h["first"]))

rng = np.random.default_rng(0)
d = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "..", "tests", "golden", "nn_known_answers.npz"))
for name in ("gauss", "lattice", "duplicates", "far", "single", "root_leaf"):
    t = d[name + "_target"]
    for (m, md) in ((10, 20), (5, 10), (3, 2), (0, 5), (100, 20)):
        check(t, m, md)
check(rng.normal(size=(20000, 3)) * [5, 5, 1], 10, 20)
check(np.round(rng.normal(size=(5000, 3)), 1), 10, 20)
