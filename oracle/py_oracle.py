"""Second, independent restatement of the reference hot path in pure Python (numpy
float32/float64 scalars, explicit loops) — TEST INFRASTRUCTURE ONLY, small cases.

It shares no code with oracle.cpp; tests/test_oracle.py checks the two against each
other so that a transcription slip in either one shows up.  PARITY UNPINNED (see
oracle.cpp header): both follow the reference source text, neither is the
reference binary.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32
f64 = np.float64


def s3(a, b, c):
    """Eigen fixed-size-3 reduction order: a0 + (a1 + a2) (float32)."""
    return f32(a + f32(b + c))


def project_point(K, r, c, d):
    """Camera.hpp:24-31."""
    fx, cx, fy, cy = (f64(K[i]) for i in (0, 2, 4, 5))
    z = f64(d) * f64(0.001)
    x = (z * (f64(c) - cx)) / fx
    y = (z * (f64(r) - cy)) / fy
    return f32(x), f32(y), f32(z)


def transform(T, p):
    """Camera.hpp:39-45 (Eigen Transform * Vector3f)."""
    T = [f32(v) for v in np.asarray(T, np.float32).reshape(12)]
    x, y, z = (f32(v) for v in p)
    return tuple(f32(T[4 * i + 3] + s3(f32(T[4 * i] * x), f32(T[4 * i + 1] * y), f32(T[4 * i + 2] * z)))
                 for i in range(3))


def inverse(T):
    """Eigen Affine3f::inverse() (3x3 cofactors)."""
    M = np.asarray(T, np.float32).reshape(3, 4)
    m = lambda i, j: f32(M[i, j])

    def cof(i, j):
        i1, i2, j1, j2 = (i + 1) % 3, (i + 2) % 3, (j + 1) % 3, (j + 2) % 3
        return f32(f32(m(i1, j1) * m(i2, j2)) - f32(m(i1, j2) * m(i2, j1)))

    c = [cof(0, 0), cof(1, 0), cof(2, 0)]
    det = s3(f32(c[0] * m(0, 0)), f32(c[1] * m(1, 0)), f32(c[2] * m(2, 0)))
    inv = f32(f32(1.0) / det)
    R = np.zeros((3, 4), np.float32)
    for j in range(3):
        R[0, j] = f32(c[j] * inv)
        R[1, j] = f32(cof(j, 1) * inv)
        R[2, j] = f32(cof(j, 2) * inv)
    for i in range(3):
        R[i, 3] = -s3(f32(R[i, 0] * m(0, 3)), f32(R[i, 1] * m(1, 3)), f32(R[i, 2] * m(2, 3)))
    return R.reshape(12)


def _c_round(v):
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)


def deproject(K, x, y, z):
    """Camera.hpp:32-38 -> (r, c); INT_MIN for NaN/overflow (x86 cvttsd2si)."""
    fx, cx, fy, cy = (f64(K[i]) for i in (0, 2, 4, 5))
    with np.errstate(all="ignore"):
        cc = (f64(x) * fx) / f64(z) + cx
        rr = (f64(y) * fy) / f64(z) + cy

    def toi(v):
        if not np.isfinite(v):
            return -2**31
        v = _c_round(float(v))
        return int(v) if -2**31 <= v < 2**31 else -2**31
    return toi(rr), toi(cc)


class Vol:
    """Volume.hpp geometry + a dense occupancy dict (insertion-ordered)."""

    def __init__(self, bounds, dims):
        self.mn = [f64(bounds[0]), f64(bounds[2]), f64(bounds[4])]
        self.mx = [f64(bounds[1]), f64(bounds[3]), f64(bounds[5])]
        # setVolumeSize then constructVolume truncation (Volume.hpp:109-128)
        self.dl = [(self.mx[a] - self.mn[a]) / f64(dims[a]) for a in range(3)]
        self.n = [int((self.mx[a] - self.mn[a]) / self.dl[a]) for a in range(3)]
        self.cells = {}  # (x,y,z) -> list of normals, insertion order = occupied_cells_

    def valid_points(self, p):
        return not any(f64(f32(p[a])) >= self.mx[a] or f64(f32(p[a])) <= self.mn[a] for a in range(3))

    def get_voxel(self, p):
        return tuple(int(math.floor((f64(f32(p[a])) - self.mn[a]) / self.dl[a])) for a in range(3))

    def valid_coords(self, c):
        return all(0 <= c[a] < self.n[a] for a in range(3))

    @staticmethod
    def hash_id(c):
        return ((c[0] << 40) ^ ((c[1] << 20) & 0xFFFFFFFFFFFFFFFF) ^ c[2]) & 0xFFFFFFFFFFFFFFFF

    def integrate(self, pts, nrm):
        """Volume.hpp:199-228."""
        for p, q in zip(pts, nrm):
            if not self.valid_points(p):
                continue
            c = self.get_voxel(p)
            if not self.valid_coords(c):
                continue
            self.cells.setdefault(c, []).append(tuple(f32(v) for v in q))

    def occupied(self):
        return [self.hash_id(c) for c in self.cells]


def degree_ok(d):
    """degree(acos(d)) in [0, 90] (CommonUtilities.hpp:17) with float acos."""
    d = f32(d)
    with np.errstate(all="ignore"):
        a = np.arccos(d)  # float32 arccos (numpy's; the C++ oracle uses glibc acosf)
    if not np.isfinite(a):
        return False
    deg = (f64(a) * 180) / 3.14159
    return 0 <= int(deg) <= 90


def reverse_ray_trace_fast(vol, K, H, W, T):
    """RayTracingEngine.hpp:136-226 (without the dead getNeighborHashes work)."""
    inv = inverse(T)
    Tm = np.asarray(T, np.float32).reshape(12)
    cc = (f32(Tm[3]), f32(Tm[7]), f32(Tm[11]))
    found, good = False, []
    for cell, normals in vol.cells.items():
        x = [f32(f64(cell[a]) * vol.dl[a] + vol.mn[a]) for a in range(3)]
        cen = [f32(f64(x[a]) + vol.dl[a] / 2.0) for a in range(3)]
        t = transform(inv, cen)
        r, c = deproject(K, *t)
        ch = vol.get_voxel(cen)
        if not (0 <= r < H and 0 <= c < W):
            continue
        d = [f32(cc[a] - cen[a]) for a in range(3)]
        s = s3(f32(d[0] * d[0]), f32(d[1] * d[1]), f32(d[2] * d[2]))
        v = [f32(d[a] / f32(np.sqrt(s))) for a in range(3)] if s > 0 else d
        collided = False
        depth = 50
        while True:
            fd = f32(depth)
            pt = [f32(cen[a] + f32(f32(v[a] * fd) / f32(1000.0))) for a in range(3)]
            depth += 1
            if not vol.valid_points(pt):
                break
            g = vol.get_voxel(pt)
            if g == ch:
                continue
            if not vol.valid_coords(g):
                break
            if g in vol.cells:
                collided = True
                break
        if not collided:
            found = True
            if 0.20 <= f64(t[2]) <= 1.0:
                for n in normals:
                    if degree_ok(s3(f32(n[0] * v[0]), f32(n[1] * v[1]), f32(n[2] * v[2]))):
                        good.append(vol.hash_id(ch))
                        break
    return found, good


def dda_cells(vol, O, E, end_inside):
    """DESIGN.md §4 exact integer DDA for one ray -> (list of missed cells, hit cell or None)."""
    go = [(f64(O[a]) - vol.mn[a]) / vol.dl[a] for a in range(3)]
    ge = [(f64(E[a]) - vol.mn[a]) / vol.dl[a] for a in range(3)]
    D = [ge[a] - go[a] for a in range(3)]
    t0, t1 = f64(0.0), f64(1.0)
    for a in range(3):
        if D[a] == 0.0:
            if go[a] < 0.0 or go[a] >= vol.n[a]:
                return [], None
        else:
            ta, tb = (f64(0.0) - go[a]) / D[a], (f64(vol.n[a]) - go[a]) / D[a]
            if ta > tb:
                ta, tb = tb, ta
            t0, t1 = max(t0, ta), min(t1, tb)
    if end_inside:
        t1 = f64(1.0)
        t0 = min(t0, f64(1.0))
    if t0 > t1:
        return [], None
    Q = 256
    clamp = lambda v, lo, hi: max(lo, min(hi, v))
    cs, ce, qs, qe = [], [], [], []
    for a in range(3):
        gs = go[a] + t0 * D[a]
        gx = ge[a] if end_inside else go[a] + t1 * D[a]
        cs.append(clamp(int(math.floor(gs)), 0, vol.n[a] - 1))
        ce.append(int(math.floor(ge[a])) if end_inside else clamp(int(math.floor(gx)), 0, vol.n[a] - 1))
        qs.append(clamp(int(math.floor(gs * Q)), cs[a] * Q, cs[a] * Q + Q - 1))
        qe.append(clamp(int(math.floor(gx * Q)), ce[a] * Q, ce[a] * Q + Q - 1))
    adq = [abs(qe[a] - qs[a]) for a in range(3)]
    st = [(ce[a] > cs[a]) - (ce[a] < cs[a]) for a in range(3)]
    # exact rational crossing times (Fraction-free: compare h_a/adq_a by cross products)
    from fractions import Fraction
    Tn = []
    for a in range(3):
        if st[a] == 0:
            Tn.append(None)
            continue
        h = 2 * ((cs[a] + 1) * Q - qs[a]) if st[a] > 0 else 2 * (qs[a] - cs[a] * Q) + 1
        Tn.append([Fraction(h, adq[a]), Fraction(2 * Q, adq[a])])
    cur = list(cs)
    steps = sum(abs(ce[a] - cs[a]) for a in range(3))
    missed = []
    for _ in range(steps):
        missed.append(tuple(cur))
        best = None
        for a in range(3):
            if Tn[a] is not None and (best is None or Tn[a][0] < Tn[best][0]):
                best = a
        cur[best] += st[best]
        Tn[best][0] += Tn[best][1]
    if end_inside:
        return missed, tuple(cur)
    return missed + [tuple(cur)], None


def will_collide(vol, a, b):
    """tests/CameraPathGen.cpp:128-156 (1 mm march a -> b; Eigen normalized())."""
    a = [f32(v) for v in a]
    b = [f32(v) for v in b]
    ab = [f32(a[i] - b[i]) for i in range(3)]
    distance = f64(f32(math.sqrt(s3(f32(ab[0] * ab[0]), f32(ab[1] * ab[1]), f32(ab[2] * ab[2])))))
    ba = [f32(b[i] - a[i]) for i in range(3)]
    sq = s3(f32(ba[0] * ba[0]), f32(ba[1] * ba[1]), f32(ba[2] * ba[2]))
    v = [f32(x / f32(math.sqrt(sq))) for x in ba] if sq > 0 else ba
    depth = 1
    while True:
        if depth > distance * 1000:
            return False
        pt = [f32(a[i] + f32(f32(v[i] * f32(depth)) / f32(1000))) for i in range(3)]
        depth += 1
        if not vol.valid_points(pt):
            continue
        c = vol.get_voxel(pt)
        if vol.valid_coords(c) and c in vol.cells:
            return True


def collision_cost_map(vol, centres):
    """tests/CameraPathGen.cpp:310-331 run_tsp: INT_MAX if willCollide else int(dist*1000)."""
    V = len(centres)
    out = np.zeros((V, V), np.int32)
    for i in range(V):
        for j in range(V):
            if will_collide(vol, centres[i], centres[j]):
                out[i, j] = 2 ** 31 - 1
            else:
                d = [f32(f32(centres[i][k]) - f32(centres[j][k])) for k in range(3)]
                out[i, j] = int(f64(f32(math.sqrt(s3(f32(d[0] * d[0]), f32(d[1] * d[1]), f32(d[2] * d[2]))))) * 1000)
    return out


def reorganized_cloud(dims, mins, res, normal, centroid, count, flags, clean):
    """OccupancyGrid.hpp:200-286 downloadReorganizedCloud restated with Python lists and
    float32 scalars (independent of oracle.cpp): x-major single-threaded order."""
    nx, ny, nz = dims
    N = nx * ny * nz
    nr = [[f32(v) for v in normal[i]] for i in range(N)]
    cr = [[f32(v) for v in centroid[i]] for i in range(N)]
    kr = [int(c) for c in count]
    occ = [False] * N
    for s in range(N):
        if not (int(flags[s]) & 1):
            continue
        if clean and kr[s] < 100:
            continue
        c = list(cr[s])
        t = []
        for a in range(3):
            q = np.floor((np.float64(c[a]) - np.float64(mins[a])) / np.float64(res[a]))
            t.append(int(q) if (np.isfinite(q) and -2147483648.0 <= q < 2147483648.0) else -2147483648)
        if not all(0 <= t[a] < dims[a] for a in range(3)):
            continue
        d = (t[0] * ny + t[1]) * nz + t[2]
        sn = list(nr[s])
        occ[d] = True
        sm = [nr[d][a] + sn[a] for a in range(3)]
        q2 = s3(sm[0] * sm[0], sm[1] * sm[1], sm[2] * sm[2])
        if q2 > f32(0):
            rt = f32(np.sqrt(q2))
            nr[d] = [sm[a] / rt for a in range(3)]
        else:
            nr[d] = sm
        if kr[d] == 0:
            cr[d] = c
        else:
            cr[d] = [(cr[d][a] + c[a]) / f32(2) for a in range(3)]
            kr[d] += 1
    out = [cr[v] + nr[v] for v in range(N) if occ[v]]
    return np.array(out, np.float32).reshape(-1, 6)
