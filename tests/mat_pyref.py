"""Second restatement of the materials extension, pure Python.

Test infrastructure only: pins oracle/rt_oracle_mat.c (the C restatement the
GPU tests compare against) on small cases with independently written code.
The book's algorithm (Ray Tracing in One Weekend v3.2, ch. 9-13) over the
counter stream; the draws come from oracle.counter_draws (the stream the
oracle's rt_oracle.c tests already pin). Python floats are IEEE binary64 and
every expression below is evaluated in the order written, without FMA, so the
result is bit-exact with a correct C restatement. Parity with the reference
itself is unpinned: the reference has no materials.
"""
import math

import numpy as np

LAMBERTIAN, METAL, DIELECTRIC = 0, 1, 2


def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _scale(t, a):
    return (t * a[0], t * a[1], t * a[2])


def _unit(a):
    return _scale(1.0 / math.sqrt(_dot(a, a)), a)


class _Stream:
    def __init__(self, oracle, seed, pixel, sample, count=8192):
        self.v = oracle.counter_draws(seed, pixel, sample, count).tolist()
        self.k = 0

    def rd(self):
        x = self.v[self.k] / 2147483648.0
        self.k += 1
        return x

    def rdr(self, lo, hi):
        return lo + (hi - lo) * self.rd()


def _hit(spheres, o, d, tmin):
    """hittable_list::hit(r, tmin, inf): (index, t) of the closest hit."""
    closest, best = math.inf, -1
    A = _dot(d, d)
    for k, (cx, cy, cz, r) in enumerate(spheres):
        amc = (o[0] - cx, o[1] - cy, o[2] - cz)
        hb = _dot(d, amc)
        c = _dot(amc, amc) - r * r
        disc = hb * hb - A * c
        if disc < 0:
            continue
        sq = math.sqrt(disc)
        t = (-hb - sq) / A
        if t < tmin or t > closest:
            t = (-hb + sq) / A
            if t < tmin or t > closest:
                continue
        closest, best = t, k
    return best, closest


def _sample(spheres, mats, lens, W, H, i, j, s, max_depth, seed, oracle):
    st = _Stream(oracle, seed, j * W + i, s)
    u = (i + st.rd()) / (W - 1)
    v = (j + st.rd()) / (H - 1)
    while True:  # random_in_unit_disk: vec3(rd(-1,1), rd(-1,1), 0), y drawn first
        y = st.rdr(-1.0, 1.0)
        x = st.rdr(-1.0, 1.0)
        if (x * x + y * y) + 0.0 * 0.0 >= 1:
            continue
        break
    lr = lens["lens_radius"]
    rx, ry = lr * x, lr * y
    lu, lv = lens["u"], lens["v"]
    off = tuple(lu[k] * rx + lv[k] * ry for k in range(3))
    base = lens["base"]
    org, llc, hor, ver = base[0], base[1], base[2], base[3]
    o = tuple(org[k] + off[k] for k in range(3))
    d = tuple((((llc[k] + u * hor[k]) + v * ver[k]) - org[k]) - off[k] for k in range(3))
    path = []
    depth = max_depth
    while True:
        if depth <= 0:
            return (0.0, 0.0, 0.0)
        idx, t = _hit(spheres, o, d, 0.001)
        if idx < 0:
            ud = _unit(d)
            tt = 0.5 * (ud[1] + 1.0)
            c = ((1.0 - tt) * 1.0 + tt * 0.5, (1.0 - tt) * 1.0 + tt * 0.7,
                 (1.0 - tt) * 1.0 + tt * 1.0)
            for a in reversed(path):
                c = (a[0] * c[0], a[1] * c[1], a[2] * c[2])
            return c
        cx, cy, cz, r = spheres[idx]
        p = tuple(o[k] + t * d[k] for k in range(3))
        out = _scale(1.0 / r, (p[0] - cx, p[1] - cy, p[2] - cz))
        front = _dot(d, out) < 0
        n = out if front else (-out[0], -out[1], -out[2])
        kind, a0, a1, a2, fuzz, ir = mats[idx]
        kind = int(kind)
        if kind == LAMBERTIAN:
            while True:
                z = st.rdr(-1.0, 1.0)
                y = st.rdr(-1.0, 1.0)
                x = st.rdr(-1.0, 1.0)
                if _dot((x, y, z), (x, y, z)) > 1:
                    continue
                break
            uv = _unit((x, y, z))
            nd = (n[0] + uv[0], n[1] + uv[1], n[2] + uv[2])
            if all(abs(e) < 1e-8 for e in nd):
                nd = n
            path.append((a0, a1, a2))
        elif kind == METAL:
            ud = _unit(d)
            dn = _dot(ud, n)
            refl = tuple(ud[k] - (2.0 * dn) * n[k] for k in range(3))
            while True:
                z = st.rdr(-1.0, 1.0)
                y = st.rdr(-1.0, 1.0)
                x = st.rdr(-1.0, 1.0)
                if _dot((x, y, z), (x, y, z)) > 1:
                    continue
                break
            f = fuzz if fuzz < 1 else 1.0
            nd = (refl[0] + f * x, refl[1] + f * y, refl[2] + f * z)
            if not _dot(nd, n) > 0:
                return (0.0, 0.0, 0.0)
            path.append((a0, a1, a2))
        else:
            ratio = (1.0 / ir) if front else ir
            ud = _unit(d)
            ct = _dot((-ud[0], -ud[1], -ud[2]), n)
            ct = ct if ct < 1.0 else 1.0
            sn = math.sqrt(1.0 - ct * ct)
            cannot = ratio * sn > 1.0
            reflect = cannot
            if not cannot:
                r0 = (1 - ratio) / (1 + ratio)
                r0 = r0 * r0
                xx = 1 - ct
                x2 = xx * xx
                reflect = r0 + (1 - r0) * ((x2 * x2) * xx) > st.rd()
            if reflect:
                dn = _dot(ud, n)
                nd = tuple(ud[k] - (2.0 * dn) * n[k] for k in range(3))
            else:
                perp = tuple(ratio * (ud[k] + ct * n[k]) for k in range(3))
                par = -math.sqrt(abs(1.0 - _dot(perp, perp)))
                nd = tuple(perp[k] + par * n[k] for k in range(3))
        o, d = p, nd
        depth -= 1


def render_mat(spheres, mats, lens, W, H, spp, max_depth, seed, oracle):
    """accum[H, W, 3] in output order (row 0 = top)."""
    spheres = [tuple(float(x) for x in row) for row in np.asarray(spheres)]
    mats = [tuple(float(x) for x in row) for row in np.asarray(mats)]
    acc = np.zeros((H, W, 3))
    for r in range(H):
        j = H - 1 - r
        for i in range(W):
            c = [0.0, 0.0, 0.0]
            for s in range(spp):
                cs = _sample(spheres, mats, lens, W, H, i, j, s, max_depth, seed, oracle)
                c = [c[0] + cs[0], c[1] + cs[1], c[2] + cs[2]]
            acc[r, i] = c
    return acc
