"""TEST INFRASTRUCTURE ONLY (never imported by the product): a restatement of the reference's photon
map (Jensen's kd-tree, reference src/libs/photon_map/pm.c) for the parity tests of the device's
photon estimate. Pinned against the reference's own dumps (tests/golden/pm_cornell_10k.npz,
tests/golden/make_pm_fixture.py): balance() must reproduce the balanced heap order and
irradiance_estimate() the reference's estimates, bit for bit.

Two forms of the k-nearest search are kept:
  * locate(): pm_locate_photons (pm.c:163-252) step by step — the kd traversal (near child first,
    the node after its children, the far child while dist1^2 < dist2[0]), the candidate array, the
    max-heap built when the (k+1)-th photon arrives and its sift-down insertion;
  * selection(): the closed form the device implements. The traversal reaches only heap indices
    whose parent is below half_stored = n/2 - 1 (pm.c:172, 372: the last two or three photons of the
    heap are never visited). The first k photons found (traversal order) fill the array; the (k+1)-th
    replaces the largest of them whatever its own distance (dist2[0] is still max_dist^2 when it is
    tested); from then on a photon enters only below the heap's maximum. The result is the k smallest
    of the reachable in-range photons except m, the largest of the first k found; m is one of the true
    k nearest exactly when the traversal finds the k nearest first, and the result is then the k
    nearest without the k-th plus the (k+1)-th.
"""
import math

import numpy as np


# ---- pm_balance (pm.c:329-494) ----
def _median_split(p, pos, start, end, median, axis):
    left, right = start, end
    while right > left:
        v = pos[p[right], axis]
        i, j = left - 1, right
        while True:
            i += 1
            while pos[p[i], axis] < v:
                i += 1
            j -= 1
            while pos[p[j], axis] > v and j > left:
                j -= 1
            if i >= j:
                break
            p[i], p[j] = p[j], p[i]
        p[i], p[right] = p[right], p[i]
        if i >= median:
            right = i - 1
        if i <= median:
            left = i + 1


def balance(pos):
    """Heap index -> stored index (1-based arrays, index 0 unused) and the split plane per heap index
    for photons pos[1..n] in stored order (pos[0] unused)."""
    n = len(pos) - 1
    pbal = np.zeros(n + 1, dtype=np.int64)
    plane = np.zeros(n + 1, dtype=np.int64)
    if n <= 1:
        pbal[1:] = np.arange(1, n + 1)
        return pbal, plane
    porg = list(range(n + 1))
    bmin = pos[1:].min(axis=0).astype(float)
    bmax = pos[1:].max(axis=0).astype(float)

    def seg(index, start, end):
        median = 1
        while 4 * median <= end - start + 1:
            median += median
        if 3 * median <= end - start + 1:
            median += median
            median += start - 1
        else:
            median = end - median + 1
        axis = 2
        ex = bmax - bmin
        if ex[0] > ex[1] and ex[0] > ex[2]:
            axis = 0
        elif ex[1] > ex[2]:
            axis = 1
        _median_split(porg, pos, start, end, median, axis)
        pbal[index] = porg[median]
        plane[index] = axis
        if median > start:
            if start < median - 1:
                tmp = bmax[axis]
                bmax[axis] = pos[porg[median], axis]
                seg(2 * index, start, median - 1)
                bmax[axis] = tmp
            else:
                pbal[2 * index] = porg[start]
        if median < end:
            if median + 1 < end:
                tmp = bmin[axis]
                bmin[axis] = pos[porg[median], axis]
                seg(2 * index + 1, median + 1, end)
                bmin[axis] = tmp
            else:
                pbal[2 * index + 1] = porg[end]

    import sys
    sys.setrecursionlimit(max(10000, sys.getrecursionlimit()))
    seg(1, 1, n)
    # leaves keep their plane from the last time they were written as a median (or 0); the search
    # only reads the planes of internal nodes
    return pbal, plane


# ---- pm_locate_photons + pm_irradiance_estimate (pm.c:91-252), step by step ----
def locate(kd_pos, kd_plane, x, max_dist, k):
    """kd_pos / kd_plane in heap order (index 0 unused). Returns (heap indices found, dist2[0])."""
    n = len(kd_pos) - 1
    half = n // 2 - 1
    dist2 = [max_dist * max_dist] + [0.0] * k
    index = [0] * (k + 1)
    st = {"found": 0, "heap": False}

    def visit(i):
        p = kd_pos[i]
        if i < half:
            ax = int(kd_plane[i])
            d1 = x[ax] - p[ax]
            if d1 > 0.0:
                visit(2 * i + 1)
                if d1 * d1 < dist2[0]:
                    visit(2 * i)
            else:
                visit(2 * i)
                if d1 * d1 < dist2[0]:
                    visit(2 * i + 1)
        d = p[0] - x[0]
        d2 = d * d
        d = p[1] - x[1]
        d2 += d * d
        d = p[2] - x[2]
        d2 += d * d
        if d2 < dist2[0]:
            if st["found"] < k:
                st["found"] += 1
                dist2[st["found"]] = d2
                index[st["found"]] = i
            else:
                f = st["found"]
                if not st["heap"]:
                    half_found = f >> 1
                    for kk in range(half_found, 0, -1):
                        parent = kk
                        ph, dst = index[kk], dist2[kk]
                        while parent <= half_found:
                            j = parent + parent
                            if j < f and dist2[j] < dist2[j + 1]:
                                j += 1
                            if dst >= dist2[j]:
                                break
                            dist2[parent] = dist2[j]
                            index[parent] = index[j]
                            parent = j
                        dist2[parent] = dst
                        index[parent] = ph
                    st["heap"] = True
                parent, j = 1, 2
                while j <= f:
                    if j < f and dist2[j] < dist2[j + 1]:
                        j += 1
                    if d2 > dist2[j]:
                        break
                    dist2[parent] = dist2[j]
                    index[parent] = index[j]
                    parent = j
                    j += j
                index[parent] = i
                dist2[parent] = d2
                dist2[0] = dist2[1]

    if n >= 1:
        visit(1)
    return index[1:st["found"] + 1], dist2[0]


def photon_dir(theta, phi):
    """pm_photon_dir (pm.c:80-86) with the tables of init_Photon_map (pm.c:61-67)."""
    a = theta * (1.0 / 256.0) * math.pi
    b = phi * (1.0 / 256.0) * math.pi
    return (math.sin(a) * math.cos(2.0 * b), math.sin(a) * math.sin(2.0 * b), math.cos(a))


def irradiance_estimate(kd, x, normal, max_dist, k, cone_k, sel=None):
    """pm_irradiance_estimate over a heap-ordered map kd (n+1 rows of pos[3], power[3], theta, phi,
    plane; row 0 unused). sel: the (heap indices, dist2[0]) of a selection; default locate()."""
    kd_pos = kd[:, 0:3]
    if sel is None:
        sel = locate(kd_pos, kd[:, 8], x, max_dist, k)
    found_idx, d0 = sel
    irr = [0.0, 0.0, 0.0]
    if len(found_idx) < 8:
        return irr, len(found_idx)
    for i in found_idx:
        p = kd_pos[i]
        dp = math.sqrt((x[0] - p[0]) * (x[0] - p[0]) + (x[1] - p[1]) * (x[1] - p[1]) + (x[2] - p[2]) * (x[2] - p[2]))
        w = 1.0 - dp / (cone_k * max_dist)
        dx, dy, dz = photon_dir(int(kd[i, 6]), int(kd[i, 7]))
        if dx * normal[0] + dy * normal[1] + dz * normal[2] < 0.0:
            irr[0] += kd[i, 3] * w
            irr[1] += kd[i, 4] * w
            irr[2] += kd[i, 5] * w
    tmp = 1.0 / ((1.0 - 2.0 / (3.0 * cone_k)) * (math.pi * d0))
    return [irr[0] * tmp, irr[1] * tmp, irr[2] * tmp], len(found_idx)


# ---- the closed form of the selection (what the device computes) ----
def traversal_before(kd_pos, kd_plane, x, a, b):
    """True when the traversal of query x visits heap node a before heap node b (a != b): the
    descendant first (a node comes after its subtree), else the side of their lowest common ancestor
    that the query's near-first order takes first."""
    da, db = a.bit_length() - 1, b.bit_length() - 1
    if da > db and (a >> (da - db)) == b:
        return True
    if db > da and (b >> (db - da)) == a:
        return False
    aa, bb = a >> max(0, da - db), b >> max(0, db - da)
    dc = min(da, db)
    while aa != bb:
        aa >>= 1
        bb >>= 1
        dc -= 1
    c = aa
    ca = a >> (da - dc - 1)  # the child of c on a's side
    ax = int(kd_plane[c])
    near = 2 * c + 1 if x[ax] - kd_pos[c][ax] > 0.0 else 2 * c
    return ca == near


def selection(kd_pos, kd_plane, x, max_dist, k):
    n = len(kd_pos) - 1
    half = n // 2 - 1
    r2 = max_dist * max_dist
    inr = []
    for i in range(1, n + 1):
        if i >= 2 and (i >> 1) >= half:
            continue  # never reached by the traversal
        p = kd_pos[i]
        d = p[0] - x[0]
        d2 = d * d
        d = p[1] - x[1]
        d2 += d * d
        d = p[2] - x[2]
        d2 += d * d
        if d2 < r2:
            inr.append((d2, i))
    if len(inr) <= k:
        return [i for _, i in inr], r2
    inr.sort()
    knn = set(i for _, i in inr[:k])
    rest = [i for _, i in inr[k:]]
    last = None  # the last of the k nearest in traversal order
    for i in knn:
        if last is None or traversal_before(kd_pos, kd_plane, x, last, i):
            last = i
    if all(traversal_before(kd_pos, kd_plane, x, last, j) for j in rest):
        chosen = [i for _, i in inr[:k - 1]] + [inr[k][1]]  # the k-th leaves, the (k+1)-th enters
        return chosen, inr[k][0]
    return [i for _, i in inr[:k]], inr[k - 1][0]
