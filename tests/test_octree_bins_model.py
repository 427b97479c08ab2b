"""The octree's quadrant-path bins (k_octree, csrc/orbx_extract.hip) as a Python model, checked
against a list restatement of ORBextractor::DistributeOctTree (ORBextractor.cc:525-733, with the
canonical (size, creation sequence) tie-break of oracle/orb_oracle.cc:391-484) on random,
clustered and sparse key sets.

The GPU parity tests compare the kernel with the C++ oracle on images; this model checks the
algorithm itself on key sets no image produces easily: thousands of random levels, keys packed
into a few pixels' neighbourhood (deep divisions, several refines per level), fewer keys than
features (every node divides down to single keys), wide frames with several initial nodes.
What the model restates, as the kernel does it:
  * the per-level path tables (orbx_geometry.cpp, Geometry::octpath): 16 x-bits of a column
    below its initial node, 16 y-bits of a row, each the comparison with DivideNode's ceil
    midpoint (ORBextractor.cc:472-473), interleaved into 2-bit digits;
  * refine: R digits below every node with > 1 key, one bin for the others, R the largest with
    nin + nact 4^R <= min(bin_cap, max(4 size, n)); the bins' exclusive prefix sums;
  * a node's child counts as differences of prefix sums over its bin range's quarters;
  * retention through the bin -> node table (max score, lowest candidate index).
The list order of the passes is the reference's (push_front of the children, erase of the
parent), so the model's output order is the reference's output order.
"""
import numpy as np
import pytest

pytestmark = []


def _midpoint(lo, hi):
    return lo + (hi - lo + 1) // 2  # halfX = ceil((float)(UR.x - UL.x) / 2)


# ------------------------------------------------------------------ reference restatement
def distribute_reference(keys, W, H, N):
    """keys: list of (x, y, score); returns the retained candidate indices in list order."""
    nini = int(np.float32(W) / np.float32(H) + np.float32(0.5))  # roundf, W/H > 0.5
    hx = np.float32(W) / np.float32(nini)
    seq = 0
    nodes = []
    for i in range(nini):
        nodes.append({"x0": int(hx * np.float32(i)), "x1": int(hx * np.float32(i + 1)),
                      "y0": 0, "y1": H, "keys": [], "seq": seq, "nomore": False})
        seq += 1
    for k, (x, y, _) in enumerate(keys):
        nodes[int(np.float32(x) / hx)]["keys"].append(k)
    lst = [n for n in nodes if n["keys"]]
    for n in lst:
        n["nomore"] = len(n["keys"]) == 1

    def divide(n):
        xm, ym = _midpoint(n["x0"], n["x1"]), _midpoint(n["y0"], n["y1"])
        ch = [{"x0": n["x0"], "x1": xm, "y0": n["y0"], "y1": ym, "keys": []},
              {"x0": xm, "x1": n["x1"], "y0": n["y0"], "y1": ym, "keys": []},
              {"x0": n["x0"], "x1": xm, "y0": ym, "y1": n["y1"], "keys": []},
              {"x0": xm, "x1": n["x1"], "y0": ym, "y1": n["y1"], "keys": []}]
        for k in n["keys"]:
            x, y, _ = keys[k]
            ch[(x >= xm) | ((y >= ym) << 1)]["keys"].append(k)
        return ch

    def push_children(n, front, rec, counter):
        nonlocal seq
        for c in divide(n):
            if not c["keys"]:
                continue
            c["seq"] = seq
            seq += 1
            c["nomore"] = len(c["keys"]) == 1
            front.insert(0, c)
            if len(c["keys"]) > 1:
                counter[0] += 1
                rec.append(c)

    finish = False
    rec = []
    while not finish:
        prev = len(lst)
        nexp = [0]
        rec = []
        front = []
        rest = []
        # the outer pass walks the list from its front; children go to the list's front
        for n in lst:
            if n["nomore"]:
                rest.append(n)
            else:
                push_children(n, front, rec, nexp)
        lst = front + rest
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + nexp[0] * 3 > N:
            while not finish:
                prev = len(lst)
                cand = sorted(rec, key=lambda n: (len(n["keys"]), n["seq"]))
                rec = []
                for n in reversed(cand):
                    front = []
                    push_children(n, front, rec, [0])
                    i = next(j for j, m in enumerate(lst) if m is n)
                    lst = front + lst[:i] + lst[i + 1:]
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    out = []
    for n in lst:
        best = n["keys"][0]
        for k in n["keys"][1:]:
            if keys[k][2] > keys[best][2]:
                best = k
        out.append(best)
    return out


# ------------------------------------------------------------------ the bins model
def path_tables(W, H):
    nini = int(np.float32(W) / np.float32(H) + np.float32(0.5))
    hx = np.float32(W) / np.float32(nini)

    def bits(c, lo, hi):
        b = 0
        for t in range(16):
            m = _midpoint(lo, hi)
            if c >= m:
                b |= 1 << (15 - t)
                lo = m
            else:
                hi = m
        return b

    def spread(v):
        return sum(((v >> i) & 1) << (2 * i) for i in range(16))

    px = []
    for x in range(W):
        i = min(int(np.float32(x) / hx), nini - 1)
        px.append(spread(bits(x, int(hx * np.float32(i)), int(hx * np.float32(i + 1)))))
    py = [spread(bits(y, 0, H)) << 1 for y in range(H)]
    return nini, hx, px, py


def distribute_bins(keys, W, H, N, bin_cap):
    """The kernel's algorithm: nodes carry (first bin, depth, digits left); the passes read child
    counts from the bins' prefix sums; the keys are swept only by refine and retention."""
    nini, hx, px, py = path_tables(W, H)
    n = len(keys)
    lab = [min(int(np.float32(x) / hx), nini - 1) for (x, _, _) in keys]  # generation 0
    cnt0 = np.bincount(lab, minlength=nini)
    seq = nini
    # node: [x0, x1, y0, y1, cnt, seq, first, depth, ls]
    lst = []
    for i in range(nini):
        if cnt0[i]:
            lst.append([int(hx * np.float32(i)), int(hx * np.float32(i + 1)), 0, H, int(cnt0[i]), i,
                        i, 0, 0])
    state = {"gen_total": nini, "bins": None, "lab": lab}

    def table():
        t = [-1] * state["gen_total"]
        for j, nd in enumerate(lst):
            t[nd[6]] = j
        last = -1
        for b in range(len(t)):
            if t[b] >= 0:
                last = t[b]
            else:
                t[b] = last
        return t

    def refine():
        t = table()
        act = [nd[4] > 1 for nd in lst]
        nact = sum(act)
        nin = len(lst) - nact
        lim = min(bin_cap, max(4 * len(lst), n))
        R = 1
        while R < 15 and nin + (nact << (2 * (R + 1))) <= lim:
            R += 1
        first = []
        tot = 0
        for a in act:
            first.append(tot)
            tot += 1 << (2 * R) if a else 1
        counts = [0] * (tot + 1)
        for k, (x, y, _) in enumerate(keys):
            j = t[state["lab"][k]]
            b = first[j]
            if act[j]:
                path = (px[x] | py[y]) << 32
                sh = 2 * (32 - lst[j][7] - R)
                b += (path >> sh) & ((1 << (2 * R)) - 1) if sh >= 0 else 0
            state["lab"][k] = b
            counts[b] += 1
        state["bins"] = np.concatenate([[0], np.cumsum(counts)]).tolist()
        state["gen_total"] = tot
        for j, nd in enumerate(lst):
            nd[6], nd[8] = first[j], (R if act[j] else 0)

    def child_counts(nd):
        E = state["bins"]
        s4 = 1 << (2 * (nd[8] - 1))
        b = nd[6]
        return [E[b + (q + 1) * s4] - E[b + q * s4] for q in range(4)]

    def children(nd, cc):
        x0, x1, y0, y1 = nd[:4]
        xm, ym = _midpoint(x0, x1), _midpoint(y0, y1)
        s4 = 1 << (2 * (nd[8] - 1))
        out = []
        for q in range(4):
            if cc[q]:
                out.append([xm if q & 1 else x0, x1 if q & 1 else xm, ym if q & 2 else y0,
                            y1 if q & 2 else ym, cc[q], None, nd[6] + q * s4, min(nd[7] + 1, 31),
                            nd[8] - 1])
        return out

    def divide(nd, cc):
        nonlocal seq
        ch = children(nd, cc)
        for c in ch:
            c[5] = seq
            seq += 1
        return ch[::-1]  # each pushed to the front: the last quadrant ends up first

    final = False
    while True:
        prev = len(lst)
        if any(nd[4] > 1 and nd[8] == 0 for nd in lst):
            refine()
        cc = {id(nd): child_counts(nd) for nd in lst if nd[4] > 1}
        if not final:
            front, rest, nexp = [], [], 0
            for nd in lst:
                if nd[4] > 1:
                    ch = divide(nd, cc[id(nd)])
                    nexp += sum(c[4] > 1 for c in ch)
                    front = ch + front
                else:
                    rest.append(nd)
            lst = front + rest
            if len(lst) >= N or len(lst) == prev:
                break
            if len(lst) + 3 * nexp > N:
                final = True
        else:
            order = sorted([nd for nd in lst if nd[4] > 1], key=lambda d: (d[4], d[5]), reverse=True)
            for nd in order:
                i = next(j for j, m in enumerate(lst) if m is nd)
                lst = divide(nd, cc[id(nd)]) + lst[:i] + lst[i + 1:]
                if len(lst) >= N:
                    break
            if len(lst) >= N or len(lst) == prev:
                break
    t = table()
    best = [None] * len(lst)
    for k, (x, y, s) in enumerate(keys):
        j = t[state["lab"][k]]
        if best[j] is None or s > keys[best[j]][2]:
            best[j] = k
    return best


def _keys(rng, W, H, n, kind):
    # keys inside the octree frame's detection area (x < W - 3, y < H - 3, as FAST cells give)
    W, H = W - 3, H - 3
    if kind == "uniform":
        pts = rng.choice(W * H, size=min(n, W * H), replace=False)
    elif kind == "cluster":  # a few tight clusters: deep divisions, several refines
        cs = []
        for _ in range(rng.integers(1, 4)):
            cx, cy = rng.integers(0, W), rng.integers(0, H)
            r = int(rng.integers(2, 12))
            xs = np.clip(cx + rng.integers(-r, r + 1, n), 0, W - 1)
            ys = np.clip(cy + rng.integers(-r, r + 1, n), 0, H - 1)
            cs.append(ys * W + xs)
        pts = np.unique(np.concatenate(cs))[:n]
        rng.shuffle(pts)
    else:  # sparse pairs: fewer keys than features, neighbours 1-3 px apart
        base = rng.choice(W * H, size=max(1, n // 2), replace=False)
        pts = np.unique(np.concatenate([base, np.clip(base + rng.integers(1, 4, base.size), 0,
                                                      W * H - 1)]))
    pts = np.sort(pts) if rng.random() < 0.5 else pts  # candidate order: cell order or any
    return [(int(p % W), int(p // W), int(rng.integers(0, 256))) for p in pts]  # (x, y, score)


@pytest.mark.parametrize("kind", ["uniform", "cluster", "sparse"])
def test_bins_model_matches_distribute_octree(kind):
    rng = np.random.default_rng({"uniform": 1, "cluster": 2, "sparse": 3}[kind])
    for it in range(60):
        H = int(rng.integers(20, 200))
        W = int(H * rng.uniform(0.6, 4.6))
        n = int(rng.integers(1, 900 if kind != "sparse" else 120))
        N = int(rng.integers(1, 300))
        keys = _keys(rng, W, H, n, kind)
        bin_cap = max(4 * (max(N + 3, 4 * 5 + 4)) + 4, int(rng.choice([64, 1024, 8192])))
        ref = distribute_reference(keys, W, H, N)
        got = distribute_bins(keys, W, H, N, bin_cap)
        assert got == ref, (kind, it, W, H, n, N, len(ref), len(got))
