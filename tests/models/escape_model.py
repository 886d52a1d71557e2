"""CPU model (oracle paths of C3): how many of psrt_trace's walked rays a
per-(sphere, direction bin) escape table would resolve without a BVH walk.

A bounce ray parks for the batched walk when, after its previous-hit sphere j
(the hint) and the big spheres, it has no hit (bt = +inf): no grid list can
bound an unbounded segment. If j's surface holds the origin and the ray's
direction lies in a cube-map bin whose cone, from apex c_j, meets no padded
BVH sphere k outside j's neighbour list (ball radius r_j + r_k + 1.5 pad),
then no BVH sphere but j's neighbours can return a root, and the ray is
decided by testing those. Rays from the ground (a big sphere) use a table
per 2-D grid column of the ground instead (apex box: the column's ground
patch). Analysis only; prints the catch rates.

    python tests/models/escape_model.py [samples] [N bins per cube face edge]
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402


def cube_bin(d, N):
    a = np.abs(d)
    f = int(np.argmax(a))
    u, v = [k for k in range(3) if k != f]
    s, t = d[u] / a[f], d[v] / a[f]
    i = min(N - 1, int((s + 1) * 0.5 * N))
    j = min(N - 1, int((t + 1) * 0.5 * N))
    return (f * 2 + (d[f] < 0)) * N * N + j * N + i


def bin_cones(N):
    """Per bin: unit axis, cos / sin of the half-angle to its corners (+1e-5 rad)."""
    axes, ca, sa = [], [], []
    for face in range(6):
        f, neg = face // 2, face % 2
        u, v = [k for k in range(3) if k != f]
        for j in range(N):
            for i in range(N):
                def direc(s, t):
                    d = np.zeros(3)
                    d[f] = -1.0 if neg else 1.0
                    d[u], d[v] = s, t
                    return d / np.linalg.norm(d)
                s0, s1 = -1 + 2 * i / N, -1 + 2 * (i + 1) / N
                t0, t1 = -1 + 2 * j / N, -1 + 2 * (j + 1) / N
                ax = direc(0.5 * (s0 + s1), 0.5 * (t0 + t1))
                cmin = min(float(ax @ direc(s, t)) for s in (s0, s1) for t in (t0, t1))
                ang = math.acos(max(-1.0, min(1.0, cmin))) + 1e-5
                axes.append(ax)
                ca.append(math.cos(ang))
                sa.append(math.sin(ang))
    return np.array(axes), np.array(ca), np.array(sa)


def cone_meets(ax, ca, sa, apex, c, R):
    """Does the cone (apex, unit axis ax, half-angle acos(ca)) meet ball(c, R)?"""
    w = c - apex
    l = float(np.linalg.norm(w))
    if l <= R * (1 + 1e-9):
        return True
    cb = float(ax @ w) / l
    if cb >= ca:
        return True
    sb = math.sqrt(max(0.0, 1 - cb * cb))
    cosd, sind = cb * ca + sb * sa, sb * ca - cb * sa
    return cosd >= 0 and sind <= R / l


def main():
    n_samples = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    oracle.build()
    sph = oracle.scene_random_spheres(1)
    cam = oracle.camera_look_at(aspect=1.5)
    r = np.abs(sph[:, 3])
    big = r > 16 * np.median(r)
    bvh = np.where(~big)[0]
    S = max(float(np.max(np.abs(sph[k, :3]) + r[k])) for k in bvh)
    pad = 2.0 ** -13 * S
    nb = {j: [k for k in bvh if k != j and np.linalg.norm(sph[j, :3] - sph[k, :3])
              <= r[j] + r[k] + 2 * pad] for j in bvh}
    axes, ca, sa = bin_cones(N)
    nbins = len(axes)
    table = {}

    def empty(j, b):
        key = (j, b)
        if key not in table:
            ok = len(nb[j]) <= 3
            if ok:
                for k in bvh:
                    if k == j or k in nb[j]:
                        continue
                    R = r[j] + r[k] + 1.5 * pad
                    if cone_meets(axes[b], ca[b], sa[b], sph[j, :3], sph[k, :3], R):
                        ok = False
                        break
            table[key] = ok
        return table[key]

    # ground table: per column cell (g x g in x, z) of the ground's surface patch
    g = 2.5 * float(np.median(r))
    gtable = {}
    gq = int(np.where(big)[0][0]) if big.any() else -1

    def gempty(o, b):
        cx, cz = math.floor(o[0] / g), math.floor(o[2] / g)
        key = (cx, cz, b)
        if key not in gtable:
            x0, z0 = cx * g, cz * g
            # the ground sphere's surface height over the patch (its top near y = c.y + r)
            cs, rs = sph[gq, :3], abs(sph[gq, 3])
            xs = [x0, x0 + g]
            zs = [z0, z0 + g]
            ys = [cs[1] + math.sqrt(max(0.0, rs * rs - (x - cs[0]) ** 2 - (z - cs[2]) ** 2))
                  for x in xs for z in zs]
            dxz = min(abs(x - cs[0]) for x in xs) if not (xs[0] <= cs[0] <= xs[1]) else 0.0
            dzz = min(abs(z - cs[2]) for z in zs) if not (zs[0] <= cs[2] <= zs[1]) else 0.0
            ytop = cs[1] + math.sqrt(max(0.0, rs * rs - dxz * dxz - dzz * dzz))
            lo = np.array([x0, min(ys) - 1e-3, z0])
            hi = np.array([x0 + g, ytop + 1e-3, z0 + g])
            m = 0.5 * (lo + hi)
            hd = float(np.linalg.norm(hi - lo)) * 0.5
            ok = True
            for k in bvh:
                if cone_meets(axes[b], ca[b], sa[b], m, sph[k, :3], r[k] + 1.5 * pad + hd):
                    ok = False
                    break
            gtable[key] = ok
        return gtable[key]

    # direction lists (r05, the material kernel's MatArgs::dl): every BVH sphere
    # the (key, bin) cone meets, up to 7, else overflow; keys: the hint sphere
    # j (apex c_j, widened by |r_j| + pad) or the 3-D cell (edge g) of a
    # ground origin (apex the cell centre, widened by half its diagonal)
    lists = {}

    def dlist(key, b, apex, wid):
        if (key, b) not in lists:
            L = []
            for k in bvh:
                if isinstance(key, int) and k == key:
                    continue
                if cone_meets(axes[b], ca[b], sa[b], apex, sph[k, :3], r[k] + 2 * pad + wid):
                    L.append(k)
                    if len(L) > 7:
                        break
            lists[(key, b)] = L if len(L) <= 7 else None
        return lists[(key, b)]
    dl_res = dl_tests = 0

    rng = np.random.default_rng(5)
    parked = caught = parked_ground = parked_bvh = gcaught = 0
    traced = 0
    for _ in range(n_samples):
        i, jj, s = rng.integers(0, 1200), rng.integers(0, 800), rng.integers(0, 100)
        _, tr = oracle.trace_sample(sph, cam, 1200, 800, i, jj, s)
        for k, b in enumerate(tr):
            if k >= 1:
                h = tr[k - 1]["index"]
                o = np.array(b["o"])
                C = float(((o - sph[h, :3]) ** 2).sum() - sph[h, 3] ** 2)
                if h >= 0 and C == 0.0:
                    break  # trapped: the device ends the path here
            traced += 1
            if k == 0:
                continue
            h = tr[k - 1]["index"]
            o, d = np.array(b["o"]), np.array(b["d"])
            # bt after the hint and the big spheres
            hits = [oracle.sphere_hit(sph[h], o, d, 0.0, np.inf)[0]] + \
                   [oracle.sphere_hit(sph[q], o, d, 0.0, np.inf)[0] for q in np.where(big)[0] if q != h]
            if any(hits):
                continue
            parked += 1
            if big[h]:
                cell = tuple(int(math.floor(o[q] / g)) for q in range(3))
                L = dlist(('c',) + cell, cube_bin(d, N), (np.array(cell, dtype=float) + 0.5) * g, 0.8661 * g)
            else:
                L = dlist(int(h), cube_bin(d, N), sph[h, :3], r[h] + pad)
            if L is not None:
                dl_res += 1
                dl_tests += len(L)
            if big[h]:
                parked_ground += 1
                if h == gq and gempty(o, cube_bin(d, N)):
                    gcaught += 1
                continue
            parked_bvh += 1
            if empty(h, cube_bin(d, N)):
                caught += 1
    print(f"samples {n_samples} traced {traced} parked(bt=inf) {parked} "
          f"from ground {parked_ground} from BVH spheres {parked_bvh}; "
          f"N={N} ({nbins} bins): caught {caught} = {caught / max(1, parked):.3f} of parked, "
          f"{caught / max(1, parked_bvh):.3f} of BVH-origin parked; table entries built {len(table)}; "
          f"ground column table: caught {gcaught} = {gcaught / max(1, parked_ground):.3f} of "
          f"ground-origin parked; total {(caught + gcaught) / max(1, parked):.3f} of parked; "
          f"direction lists (<= 7) resolve {dl_res / max(1, parked):.3f} of parked, "
          f"mean list {dl_tests / max(1, dl_res):.2f}")


if __name__ == "__main__":
    main()
