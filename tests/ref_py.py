"""Independent pure-Python/numpy restatements used to cross-check the C++
oracle (test infrastructure only).  Written from the reference's behaviour
(orb_extractor.cc) and SURVEY.md Appendix A, separately from oracle/*.cc, so a
transcription slip in either shows up as a mismatch.  Small inputs only."""
from __future__ import annotations

import numpy as np

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3),
          (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def fast_score_def(img: np.ndarray, y: int, x: int) -> int:
    """max over the 16 nine-pixel arcs of min(v - p) / min(p - v), minus 1."""
    v = int(img[y, x])
    d = [v - int(img[y + dy, x + dx]) for dx, dy in CIRCLE]
    best = -10**9
    for s in range(16):
        arc = [d[(s + k) % 16] for k in range(9)]
        best = max(best, min(arc), min(-a for a in arc))
    return best - 1


def fast_nms_def(roi: np.ndarray, th: int):
    """cv::FAST(roi, th, nonmax=true) by definition: corners at th in
    [3, rows-3) x [3, cols-3), strict 3x3 maximum of the in-ROI score map."""
    rows, cols = roi.shape
    S = np.zeros((rows, cols), np.int64)
    for y in range(3, rows - 3):
        for x in range(3, cols - 3):
            s = fast_score_def(roi, y, x)
            if s >= th:
                S[y, x] = s
    out = []
    for y in range(3, rows - 3):
        for x in range(3, cols - 3):
            s = S[y, x]
            if s == 0:
                continue
            nb = S[y - 1:y + 2, x - 1:x + 2].copy()
            nb[1, 1] = -1
            if s > nb.max():
                out.append((x, y, int(s)))
    return out


def resize_linear(src: np.ndarray, dw: int, dh: int, rounding: str = "sse") -> np.ndarray:
    """cv::resize INTER_LINEAR for 8UC1, vectorised.
    rounding "sse": the 128-bit SIMD body's rounding on x < the block end,
    the scalar tail after; "scalar": every column the scalar rounding."""
    sh, sw = src.shape
    sx_scale = 1.0 / (dw / sw)
    sy_scale = 1.0 / (dh / sh)
    dx = np.arange(dw)
    fx = ((dx + 0.5) * sx_scale - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    neg = sx < 0
    fx[neg], sx[neg] = 0, 0
    right = sx + 1 >= sw
    xmax = int(np.argmax(right)) if right.any() else dw
    clamp = sx >= sw - 1
    fx[clamp], sx[clamp] = 0, sw - 1
    a0 = np.clip(np.rint((np.float32(1) - fx) * np.float32(2048)), -32768, 32767).astype(np.int64)
    a1 = np.clip(np.rint(fx * np.float32(2048)), -32768, 32767).astype(np.int64)

    dy = np.arange(dh)
    fy = ((dy + 0.5) * sy_scale - 0.5).astype(np.float32)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy.astype(np.float32)).astype(np.float32)
    b0 = np.clip(np.rint((np.float32(1) - fy) * np.float32(2048)), -32768, 32767).astype(np.int64)
    b1 = np.clip(np.rint(fy * np.float32(2048)), -32768, 32767).astype(np.int64)
    r0 = np.clip(sy, 0, sh - 1)
    r1 = np.clip(sy + 1, 0, sh - 1)

    S = src.astype(np.int64)
    sx1 = np.minimum(sx + 1, sw - 1)

    def hres(rows):
        H = S[rows][:, sx] * a0 + S[rows][:, sx1] * a1
        H[:, xmax:] = S[rows][:, sx[xmax:]] * 2048
        return H

    H0, H1 = hres(r0), hres(r1)
    B0, B1 = b0[:, None], b1[:, None]
    # SIMD body: x <= w-16 in 16s, then x < w-8 in 8s
    x = 0
    while x <= dw - 16:
        x += 16
    while x < dw - 8:
        x += 8
    vec_end = x if rounding == "sse" else 0

    def s16(a):
        return np.clip(a, -32768, 32767)

    m0 = (s16(H0 >> 4) * B0) >> 16
    m1 = (s16(H1 >> 4) * B1) >> 16
    vec = np.clip((s16(m0 + m1) + 2) >> 2, 0, 255)
    sca = np.clip((H0 * B0 + H1 * B1 + (1 << 21)) >> 22, 0, 255)
    out = sca.copy()
    out[:, :vec_end] = vec[:, :vec_end]
    return out.astype(np.uint8)


def gauss7(src: np.ndarray) -> np.ndarray:
    k = np.array([18, 34, 48, 56, 48, 34, 18], np.int64)
    h, w = src.shape

    def refl(i, n):
        i = np.abs(i)
        return np.where(i >= n, 2 * n - 2 - i, i)

    xs = refl(np.arange(w)[:, None] + np.arange(-3, 4)[None, :], w)
    ys = refl(np.arange(h)[:, None] + np.arange(-3, 4)[None, :], h)
    S = src.astype(np.int64)
    Hs = (S[:, xs] * k).sum(-1)             # h x w
    V = (Hs[ys] * k[None, :, None]).sum(1)  # h x w
    return np.minimum((V + (1 << 15)) >> 16, 255).astype(np.uint8)


def distribute_octree(kps, min_x, max_x, min_y, max_y, n_feats):
    """DistributeOctTree (orb_extractor.cc:542-742) with Python lists standing
    in for std::list; kps = [(x, y, response)] in to_dist order.  Returns the
    kept keypoints in node-list order."""
    r = float(np.float32(max_x - min_x) / np.float32(max_y - min_y))
    n_ini = int(np.floor(r + 0.5))  # std::round: half away from zero
    hx = np.float32(max_x - min_x) / np.float32(n_ini)

    class Node:
        __slots__ = ("ul", "ur", "bl", "br", "kps", "no_more")

        def __init__(self):
            self.kps, self.no_more = [], False

    def divide(nd):
        half_x = int(np.ceil(np.float32(nd.ur[0] - nd.ul[0]) / np.float32(2)))
        half_y = int(np.ceil(np.float32(nd.br[1] - nd.ul[1]) / np.float32(2)))
        c = [Node() for _ in range(4)]
        c[0].ul, c[0].ur = nd.ul, (nd.ul[0] + half_x, nd.ul[1])
        c[0].bl, c[0].br = (nd.ul[0], nd.ul[1] + half_y), (nd.ul[0] + half_x, nd.ul[1] + half_y)
        c[1].ul, c[1].ur, c[1].bl, c[1].br = c[0].ur, nd.ur, c[0].br, (nd.ur[0], nd.ul[1] + half_y)
        c[2].ul, c[2].ur, c[2].bl, c[2].br = c[0].bl, c[0].br, nd.bl, (c[0].br[0], nd.bl[1])
        c[3].ul, c[3].ur, c[3].bl, c[3].br = c[2].ur, c[1].br, c[2].br, nd.br
        for kp in nd.kps:
            if kp[0] < c[0].ur[0]:
                (c[0] if kp[1] < c[0].br[1] else c[2]).kps.append(kp)
            else:
                (c[1] if kp[1] < c[0].br[1] else c[3]).kps.append(kp)
        for ch in c:
            if len(ch.kps) == 1:
                ch.no_more = True
        return c

    nodes = []
    roots = []
    for i in range(n_ini):
        n = Node()
        x0 = int(hx * np.float32(i))
        x1 = int(hx * np.float32(i + 1))
        n.ul, n.ur, n.bl, n.br = (x0, 0), (x1, 0), (x0, max_y - min_y), (x1, max_y - min_y)
        nodes.append(n)
        roots.append(n)
    for kp in kps:
        roots[int(np.float32(kp[0]) / hx)].kps.append(kp)
    nodes = [n for n in nodes if n.kps]
    for n in nodes:
        if len(n.kps) == 1:
            n.no_more = True

    finished = False
    expand = []
    while not finished:
        prev = len(nodes)
        front = []  # pushed to the list front, newest first
        expand = []
        keep = []
        for n in nodes:
            if n.no_more:
                keep.append(n)
                continue
            for ch in divide(n):
                if ch.kps:
                    front.insert(0, ch)
                    if len(ch.kps) > 1:
                        expand.append(ch)
        nodes = front + keep
        if len(nodes) >= n_feats or len(nodes) == prev:
            finished = True
        elif len(nodes) + 3 * len(expand) > n_feats:
            while not finished:
                prev = len(nodes)
                order = sorted(range(len(expand)), key=lambda j: (len(expand[j].kps), expand[j].ul[0], j))
                cand = [expand[j] for j in order]
                expand = []
                for nd in reversed(cand):
                    kids = [ch for ch in divide(nd) if ch.kps]
                    pos = next(i for i, m in enumerate(nodes) if m is nd)
                    del nodes[pos]
                    for ch in kids:
                        nodes.insert(0, ch)
                        if len(ch.kps) > 1:
                            expand.append(ch)
                    if len(nodes) >= n_feats:
                        break
                if len(nodes) >= n_feats or len(nodes) == prev:
                    finished = True
    out = []
    for n in nodes:
        best = n.kps[0]
        for kp in n.kps[1:]:
            if kp[2] > best[2]:
                best = kp
        out.append(best)
    return out


def stereo_match_py(kl, dl, kr, dr, pyr_l, pyr_r, scale, inv_scale, bf, mb):
    """Frame::ComputeStereoMatches (frame.cc:828-986) restated with numpy float32
    scalars: per left keypoint the row band candidates, Hamming best (first
    strict minimum), 11x11 L1 sweep on reflect-101 padded levels, parabola,
    disparity clamp, then the 1.5 * 1.4 * median filter.  -> (uright, depth)."""
    f32 = np.float32
    nl = len(kl)
    ur = np.full(nl, -1.0, np.float32)
    dep = np.full(nl, -1.0, np.float32)
    rows = pyr_l[0].shape[0]
    bits = np.unpackbits(np.arange(256, dtype=np.uint8)[:, None], axis=1).sum(1)
    table = [[] for _ in range(rows)]
    for i in range(len(kr)):
        y = f32(kr["y"][i])
        r = f32(2.0) * f32(scale[kr["octave"][i]])
        for yi in range(int(np.floor(f32(y - r))), int(np.ceil(f32(y + r))) + 1):
            if 0 <= yi < rows:
                table[yi].append(i)
    maxD = f32(f32(bf) / f32(mb))
    pads = [(np.pad(a, 19, mode="reflect").astype(np.int64), np.pad(b, 19, mode="reflect").astype(np.int64))
            for a, b in zip(pyr_l, pyr_r)]
    kept = []
    for i in range(nl):
        uL, vL, oct_ = f32(kl["x"][i]), f32(kl["y"][i]), int(kl["octave"][i])
        row = int(vL)
        if row >= rows or not table[row]:
            continue
        minU = f32(uL - maxD)
        if uL < 0:
            continue
        best, bidx = 100, 0
        for j in table[row]:
            if abs(int(kr["octave"][j]) - oct_) > 1:
                continue
            uR = f32(kr["x"][j])
            if minU <= uR <= uL:
                d = int(bits[np.bitwise_xor(dl[i], dr[j])].sum())
                if d < best:
                    best, bidx = d, j
        if best >= 75:
            continue
        inv = f32(inv_scale[oct_])
        # std::round: half away from zero (coordinates are >= 0)
        su = f32(np.floor(np.float64(f32(uL * inv)) + 0.5))
        sv = f32(np.floor(np.float64(f32(vL * inv)) + 0.5))
        sr = f32(np.floor(np.float64(f32(f32(kr["x"][bidx]) * inv)) + 0.5))
        if sr < 0 or f32(sr + 11) >= pyr_l[oct_].shape[1]:
            continue
        PL, PR = pads[oct_]
        xl, yl, xr = int(su) + 19, int(sv) + 19, int(sr) + 19
        wl = PL[yl - 5:yl + 6, xl - 5:xl + 6]
        ds = [int(np.abs(wl - PR[yl - 5:yl + 6, xr + inc - 5:xr + inc + 6]).sum()) for inc in range(-5, 6)]
        bi = int(np.argmin(ds))  # first minimum
        if bi in (0, 10):
            continue
        d1, d2, d3 = f32(ds[bi - 1]), f32(ds[bi]), f32(ds[bi + 1])
        delta = f32(f32(d1 - d3) / f32(f32(2.0) * f32(f32(d1 + d3) - f32(f32(2.0) * d2))))
        if not (-1 <= delta <= 1):
            continue
        bu = f32(f32(scale[oct_]) * f32(f32(sr + f32(bi - 5)) + delta))
        disp = f32(uL - bu)
        if f32(0) <= disp < maxD:
            if disp <= 0:
                disp = f32(0.01)
                bu = f32(np.float64(uL) - 0.01)
            dep[i] = f32(f32(bf) / disp)
            ur[i] = bu
            kept.append((ds[bi], i))
    if kept:
        kept.sort()
        th = f32(f32(f32(1.5) * f32(1.4)) * f32(kept[len(kept) // 2][0]))
        for d, i in kept:
            if not (f32(d) < th):
                ur[i] = dep[i] = -1.0
    return ur, dep


# --- ORBmatcher projection searches (orb_matcher.cc, frame.cc) --------------
# Float arithmetic in float32 with the reference build's fused multiply-adds;
# fmaf is emulated in x86 long double (64-bit mantissa: the product of two
# floats is exact, the sum rounds once before the final float rounding).

def _f(x):
    return np.float32(x)


def _fmaf(a, b, c):
    return np.float32(np.longdouble(np.float32(a)) * np.longdouble(np.float32(b))
                      + np.longdouble(np.float32(c)))


def _cross(a, b):
    return [_fmaf(a[1], b[2], -(_f(a[2]) * _f(b[1]))), _fmaf(a[2], b[0], -(_f(a[0]) * _f(b[2]))),
            _fmaf(a[0], b[1], -(_f(a[1]) * _f(b[0])))]


def _qrot(q, p):
    qv = [q[0], q[1], q[2]]
    uv = _cross(qv, p)
    uv = [_f(u + u) for u in uv]
    c = _cross(qv, uv)
    return [_f(_fmaf(q[3], uv[i], p[i]) + c[i]) for i in range(3)]


def _se3(T, p):
    r = _qrot([_f(v) for v in T[:4]], [_f(v) for v in p])
    return [_f(r[i] + _f(T[4 + i])) for i in range(3)]


def _round(v):
    """std::round / roundf: half away from zero."""
    v = float(v)
    return int(np.trunc(v + np.copysign(0.5, v)))


def _popcount_dist(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


class _PyFrame:
    def __init__(self, geom, kps, desc, uright, claimed):
        self.g, self.kps, self.desc, self.ur = geom, kps, desc, uright
        self.inv_w = _f(_f(64) / _f(_f(geom.max_x) - _f(geom.min_x)))
        self.inv_h = _f(_f(48) / _f(_f(geom.max_y) - _f(geom.min_y)))
        n = len(kps)
        self.holder = [-1] * n
        self.hobs = [False] * n
        if claimed is not None:
            for i in range(n):
                if claimed[i]:
                    self.holder[i], self.hobs[i] = -2, True
        self.grid = {}
        for i in range(n):
            px = _round(_f(_f(kps["x"][i]) - _f(geom.min_x)) * self.inv_w)
            py = _round(_f(_f(kps["y"][i]) - _f(geom.min_y)) * self.inv_h)
            if 0 <= px < 64 and 0 <= py < 48:
                self.grid.setdefault((px, py), []).append(i)

    def area(self, x, y, r, lo, hi):
        x, y, r = _f(x), _f(y), _f(r)
        g = self.g
        x0 = max(0, int(np.floor(_f(_f(x - _f(g.min_x)) - r) * self.inv_w)))
        if x0 >= 64:
            return []
        x1 = min(63, int(np.ceil(_f(_f(x - _f(g.min_x)) + r) * self.inv_w)))
        if x1 < 0:
            return []
        y0 = max(0, int(np.floor(_f(_f(y - _f(g.min_y)) - r) * self.inv_h)))
        if y0 >= 48:
            return []
        y1 = min(47, int(np.ceil(_f(_f(y - _f(g.min_y)) + r) * self.inv_h)))
        if y1 < 0:
            return []
        chk = lo >= 0 or hi >= 0
        out = []
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for i in self.grid.get((ix, iy), []):
                    o = int(self.kps["octave"][i])
                    if chk and (o < lo or (hi >= 0 and o > hi)):
                        continue
                    if abs(_f(self.kps["x"][i]) - x) < r and abs(_f(self.kps["y"][i]) - y) < r:
                        out.append(i)
        return out

    def blocked(self, i):
        return self.holder[i] != -1 and self.hobs[i]


def search_last_py(geom, cam, mb, Tcw, Tlw, kps, desc, uright, claimed, pts, th, mono, check_ori):
    """SearchByProjection(CurrentFrame, LastFrame) (orb_matcher.cc:1518-1728)."""
    F = _PyFrame(geom, kps, desc, uright, claimed)
    fx, fy, cx, cy, bf = (_f(v) for v in cam)
    # Tcw.inverse().translation(): conjugate quaternion renormalised, then -t rotated
    q = [-_f(Tcw[0]), -_f(Tcw[1]), -_f(Tcw[2]), _f(Tcw[3])]
    s = _f(_f(_f(q[0] * q[0]) + _f(q[2] * q[2])) + _f(_f(q[1] * q[1]) + _f(q[3] * q[3])))
    ln = np.sqrt(s, dtype=np.float32)
    q = [_f(c / ln) for c in q]
    twc = _qrot(q, [-_f(Tcw[4]), -_f(Tcw[5]), -_f(Tcw[6])])
    tlc = _se3(Tlw, twc)
    fwd = tlc[2] > _f(mb) and not mono
    bwd = -tlc[2] > _f(mb) and not mono
    hist = [[] for _ in range(30)]
    nm = 0
    th = _f(th)
    for j, P in enumerate(pts):
        X = _se3(Tcw, P["Xw"])
        invz = _f(1.0 / float(X[2]))
        if invz < 0:
            continue
        u = _f(_f(fx * X[0]) / X[2] + cx)
        v = _f(_f(fy * X[1]) / X[2] + cy)
        if u < _f(geom.min_x) or u > _f(geom.max_x) or v < _f(geom.min_y) or v > _f(geom.max_y):
            continue
        o = int(P["octave"])
        rad = _f(th * _f(geom.scale_factors[o]))
        if fwd:
            cand = F.area(u, v, rad, o, -1)
        elif bwd:
            cand = F.area(u, v, rad, 0, o)
        else:
            cand = F.area(u, v, rad, o - 1, o + 1)
        best, bi = 256, -1
        for i in cand:
            if F.blocked(i):
                continue
            if uright is not None and uright[i] > 0:
                ur = _fmaf(-bf, invz, u)
                if abs(_f(ur - _f(uright[i]))) > rad:
                    continue
            d = _popcount_dist(P["desc"], desc[i])
            if d < best:
                best, bi = d, i
        if best <= 100:
            F.holder[bi], F.hobs[bi] = j, bool(P["has_obs"])
            nm += 1
            if check_ori:
                rot = _f(_f(P["angle"]) - _f(kps["angle"][bi]))
                if rot < 0:
                    rot = _f(rot + _f(360))
                b = _round(_f(rot * _f(_f(30) / _f(360))))
                hist[0 if b == 30 else b].append(bi)
    nulled = set()
    if check_ori:
        sizes = [len(h) for h in hist]
        order = sorted(range(30), key=lambda b: (-sizes[b], b))
        m1 = sizes[order[0]]
        keep = {order[0]} if m1 > 0 else set()
        if m1 > 0 and sizes[order[1]] > 0 and not (_f(sizes[order[1]]) < _f(0.1) * _f(m1)):
            keep.add(order[1])
            if sizes[order[2]] > 0 and not (_f(sizes[order[2]]) < _f(0.1) * _f(m1)):
                keep.add(order[2])
        for b in range(30):
            if b not in keep:
                for i in hist[b]:
                    F.holder[i] = -1
                    nulled.add(i)
                    nm -= 1
    match = np.array([-2 if i in nulled else (h if h >= 0 else -1)
                      for i, h in enumerate(F.holder)], np.int32)
    return nm, match


def search_local_py(geom, kps, desc, uright, claimed, pts, views, th, nn):
    """SearchByProjection(F, vpMapPoints, th) (orb_matcher.cc:42-137)."""
    F = _PyFrame(geom, kps, desc, uright, claimed)
    nm = 0
    for j, (P, V) in enumerate(zip(pts, views)):
        if not V["in_view"]:
            continue
        lv = int(V["level"])
        r = _f(2.5) if float(V["view_cos"]) > 0.998 else _f(4.0)
        if th != 1.0:
            r = _f(r * _f(th))
        rs = _f(r * _f(geom.scale_factors[lv]))
        cand = F.area(V["proj_x"], V["proj_y"], rs, lv - 1, lv)
        ranked = []
        for pos, i in enumerate(cand):
            if F.blocked(i):
                continue
            if uright is not None and uright[i] > 0 and abs(_f(_f(V["proj_xr"]) - _f(uright[i]))) > rs:
                continue
            ranked.append((_popcount_dist(P["desc"], desc[i]), pos, i))
        if not ranked:
            continue
        ranked.sort()
        d1, _, i1 = ranked[0]
        d2, l2 = (ranked[1][0], int(kps["octave"][ranked[1][2]])) if len(ranked) > 1 else (256, -1)
        if d1 > 100:
            continue
        if int(kps["octave"][i1]) == l2 and _f(d1) > _f(_f(nn) * _f(d2)):
            continue
        F.holder[i1], F.hobs[i1] = j, bool(P["flags"] & 2)
        nm += 1
    return nm, np.array([h if h >= 0 else -1 for h in F.holder], np.int32)


def _three_maxima_keep(hist):
    sizes = [len(h) for h in hist]
    order = sorted(range(30), key=lambda b: (-sizes[b], b))
    m1 = sizes[order[0]]
    keep = {order[0]} if m1 > 0 else set()
    if m1 > 0 and sizes[order[1]] > 0 and not (_f(sizes[order[1]]) < _f(0.1) * _f(m1)):
        keep.add(order[1])
        if sizes[order[2]] > 0 and not (_f(sizes[order[2]]) < _f(0.1) * _f(m1)):
            keep.add(order[2])
    return keep


def _rot_bin(a_ref, a_cur):
    rot = _f(_f(a_ref) - _f(a_cur))
    if rot < 0:
        rot = _f(rot + _f(360))
    b = _round(_f(rot * _f(_f(30) / _f(360))))
    return 0 if b == 30 else b


def search_kf_py(geom, cam, Tcw, kps, desc, claimed, pts, angles, th, orb_dist, check_ori):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
    (orb_matcher.cc:1730-1839): every keypoint holding a point is skipped."""
    import binding as orc  # the restated PredictScale of the oracle (pinned separately)

    F = _PyFrame(geom, kps, desc, None, claimed)
    fx, fy, cx, cy = (_f(v) for v in cam[:4])
    q = [-_f(Tcw[0]), -_f(Tcw[1]), -_f(Tcw[2]), _f(Tcw[3])]
    s = _f(_f(_f(q[0] * q[0]) + _f(q[2] * q[2])) + _f(_f(q[1] * q[1]) + _f(q[3] * q[3])))
    ln = np.sqrt(s, dtype=np.float32)
    q = [_f(c / ln) for c in q]
    Ow = _qrot(q, [-_f(Tcw[4]), -_f(Tcw[5]), -_f(Tcw[6])])
    hist = [[] for _ in range(30)]
    nm = 0
    th = _f(th)
    for j, P in enumerate(pts):
        if P["flags"] & 1:
            continue
        X = [_f(v) for v in P["Xw"]]
        Xc = _se3(Tcw, X)
        u = _f(_f(fx * Xc[0]) / Xc[2] + cx)
        v = _f(_f(fy * Xc[1]) / Xc[2] + cy)
        if u < _f(geom.min_x) or u > _f(geom.max_x) or v < _f(geom.min_y) or v > _f(geom.max_y):
            continue
        PO = [_f(X[i] - Ow[i]) for i in range(3)]
        d3 = np.sqrt(_fmaf(PO[2], PO[2], _fmaf(PO[0], PO[0], _f(PO[1] * PO[1]))), dtype=np.float32)
        if d3 < _f(_f(0.8) * _f(P["min_dist"])) or d3 > _f(_f(1.2) * _f(P["max_dist"])):
            continue
        lv = orc.predict_scale(P["max_dist"], d3, geom.log_scale_factor, geom.n_levels)
        rad = _f(th * _f(geom.scale_factors[lv]))
        cand = F.area(u, v, rad, lv - 1, lv + 1)
        best, bi = 256, -1
        for i in cand:
            if F.holder[i] != -1:
                continue
            d = _popcount_dist(P["desc"], desc[i])
            if d < best:
                best, bi = d, i
        if best <= orb_dist:
            F.holder[bi], F.hobs[bi] = j, True
            nm += 1
            if check_ori:
                hist[_rot_bin(angles[j], kps["angle"][bi])].append(bi)
    nulled = set()
    if check_ori:
        keep = _three_maxima_keep(hist)
        for b in range(30):
            if b not in keep:
                for i in hist[b]:
                    F.holder[i] = -1
                    nulled.add(i)
                    nm -= 1
    return nm, np.array([-2 if i in nulled else (h if h >= 0 else -1)
                         for i, h in enumerate(F.holder)], np.int32)


def search_bow_py(kf_fv, kf_desc, kf_angle, kf_valid, f_fv, f_desc, f_angle, nn, check_ori):
    """SearchByBoW(pKF, F) (orb_matcher.cc:215-389) over two FeatureVectors given
    as dicts node -> [feature indices]: the common nodes in ascending order."""
    match = [-1] * len(f_desc)
    hist = [[] for _ in range(30)]
    nm = 0
    for node in sorted(set(kf_fv) & set(f_fv)):
        for ik in kf_fv[node]:
            if not kf_valid[ik]:
                continue
            ranked = [(_popcount_dist(kf_desc[ik], f_desc[i]), pos, i)
                      for pos, i in enumerate(f_fv[node]) if match[i] < 0]
            if not ranked:
                continue
            ranked.sort()
            d1, _, i1 = ranked[0]
            d2 = ranked[1][0] if len(ranked) > 1 else 256
            if d1 <= 50 and _f(d1) < _f(_f(nn) * _f(d2)):
                match[i1] = ik
                nm += 1
                if check_ori:
                    hist[_rot_bin(kf_angle[ik], f_angle[i1])].append(i1)
    if check_ori:
        keep = _three_maxima_keep(hist)
        for b in range(30):
            if b not in keep:
                for i in hist[b]:
                    match[i] = -1
                    nm -= 1
    return nm, np.array(match, np.int32)


# --- DBoW2 transform (TemplatedVocabulary.h:1057-1179) -----------------------
def load_vocab_py(path):
    """loadFromTextFile restated in Python: nodes as dicts."""
    lines = open(path).read().split("\n")
    k, L, sc, wt = (int(x) for x in lines[0].split())
    nodes = [dict(parent=0, children=[], desc=bytes(32), weight=0.0, word=0)]
    n_words = 0
    for line in lines[1:]:  # every getline after the header, the empty last one included
        tok = line.split()
        pid = int(tok[0]) if tok else 0
        leaf = int(tok[1]) if len(tok) > 1 else 0
        desc = bytes(int(x) & 255 for x in tok[2:34]) if len(tok) >= 34 else bytes(32)
        w = float(tok[34]) if len(tok) > 34 else 0.0
        nid = len(nodes)
        nodes.append(dict(parent=pid, children=[], desc=desc, weight=w, word=0))
        nodes[pid]["children"].append(nid)
        if leaf > 0:
            nodes[nid]["word"] = n_words
            n_words += 1
    return dict(k=k, L=L, scoring=sc, weighting=wt, nodes=nodes, words=n_words)


def bow_transform_py(V, descs, levelsup):
    nodes = V["nodes"]
    bow, fv = {}, {}
    if V["words"] == 0:
        return bow, fv
    tf = V["weighting"] in (0, 1)
    for i, d in enumerate(np.asarray(descs, np.uint8)):
        cur, nid, level = 0, 0, 0
        while True:
            level += 1
            ch = nodes[cur]["children"]
            dists = [int(np.unpackbits(np.bitwise_xor(d, np.frombuffer(nodes[c]["desc"], np.uint8))).sum())
                     for c in ch]
            cur = ch[int(np.argmin(dists))]  # argmin: first minimum
            if level == V["L"] - levelsup:
                nid = cur
            if not nodes[cur]["children"]:
                break
        w = nodes[cur]["weight"]
        if not w > 0:
            continue
        word = nodes[cur]["word"]
        if word in bow:
            if tf:
                bow[word] += w
        else:
            bow[word] = w
        fv.setdefault(nid, []).append(i)
    bow = dict(sorted(bow.items()))
    if V["scoring"] != 5:
        if V["scoring"] == 1:
            norm = 0.0
            for x in bow.values():
                norm = float(np.longdouble(x) * np.longdouble(x) + np.longdouble(norm))
            norm = np.sqrt(norm)
        else:
            norm = 0.0
            for x in bow.values():
                norm += abs(x)
        if norm > 0:
            bow = {k: x / norm for k, x in bow.items()}
    elif tf and bow:
        nd = float(len(bow))
        bow = {k: x / nd for k, x in bow.items()}
    return bow, dict(sorted(fv.items()))
