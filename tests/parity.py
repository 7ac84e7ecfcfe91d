"""End-to-end parity contract of one HRegNet forward against a reference result
(BASELINE.json north_star), shared by the oracle and the GPU tests.

A forward is a chain of discrete selections (FPS / WFPS, kNN) and continuous maps between
them.  Two correct fp32 implementations agree on every selection except where two
candidates are tied to within fp32 rounding, and there a selection may go either way; the
reference's own CPU fp32 run and ours both sit ~1e-6 (relative) from the exact values.
So the contract is:

* level-1 FPS indices bit-exact (input-only); every kNN and WFPS selection equal to the
  reference's -- compared by the points selected, not by index, since a flip upstream
  permutes a level's keypoints -- EXCEPT where the mismatch is a float64 near tie on the
  reference's own inputs: a WFPS run's first divergence with relative margin
  <= WFPS_TIE, or a kNN row whose k-th / (k+1)-th distances differ by <= KNN_TIE
  relative, or a selection downstream of an earlier mismatch (its inputs moved);
* every continuous output (keypoints, sigma, descriptors, correspondences, weights) on
  the rows NOT downstream of a selection mismatch, normalised (max |a - b| / max |b| over
  the tensor): against the reference's float64 replay on its own selections (fixtures
  made by make_golden.py carry one) within max(FEAT_TOL = 1e-5, SPREAD x the fp32
  reference's own distance from float64, pooled per quantity over the committed fixtures
  -- up to 4.8e-5 at level 3), and against a plain fp32 result (the CPU oracle) within
  twice that;
* R / t within RT_TOL absolute everywhere (north_star: 1e-4);
* the comparison may not shrink its own sample: at every level and head at least ROWS_FLOOR
  of the rows are compared (not downstream of a selection mismatch).

report() prints the observed numbers and, when HREG_PARITY_REPORT names a file, appends them
there (the GPU run's evidence, committed under profiles/).

Inputs are dicts in the fixture layout of tests/golden/make_golden.py (as_layout converts
an engine / oracle result): src, dst [B,N,3]; {src,dst}_{xyz,sigmas,desc,fps}_{1,2,3}
(desc [B,C,M]); R{l}, t{l}; corres_{l}, weights_{l}; knn_<site> [B,M,k] for the sites of
KNN_NAMES (make_golden TRAIN_KNN_NAMES order).
"""
from __future__ import annotations

import os

import numpy as np

WFPS_TIE = 2e-5   # the largest relative sigma error we measure upstream is ~1e-5
KNN_TIE = 1e-5
FEAT_TOL = 1e-5   # A6-A13 outputs at <= 1e-5 relative
SPREAD = 4.0      # ... or SPREAD x the fp32 reference's own distance from float64 (as the
#                   training-gradient bars, test_gpu_train_graph.py)
SPREAD_FIXTURES = ("hregnet_lidar_b2_n4096.npz", "hregnet_cube_b1_n16384.npz",
                   "model_v2_lidar_b2_n4096.npz", "model_v2_lidar_b1_n65536.npz")
RT_TOL = 1e-4
KP_TOL = 1e-3     # "the same point" when matching selections across implementations
# The comparison may not shrink its own sample.  Two bounds:
# * the root selection mismatches (near ties that are not downstream of another mismatch) at
#   most max(ROOT_MIN, ROOT_FRAC x rows) per site -- many near-tie flips are a defect, not luck;
# * the rows compared at every level and head at least ROWS_FLOOR.  One root tie does reach
#   further than its own rows: a level-2 WFPS tie of 2 points moves every level-3 group that
#   holds one of them (18 of 256 rows on hregnet_cube_b1_n16384, the CPU oracle: 93 %).
ROOT_MIN, ROOT_FRAC = 4, 0.01
ROWS_FLOOR = 0.9
# ... except the CoarseReg head (level 3), two neighbourhood hops below the level-3 WFPS: one
# flipped dst keypoint moves the neighbour-aware descriptors of its k = 8 spatial neighbours
# (layers.py:315-362), and every src keypoint with one of those among its k = 8 descriptor
# neighbours (layers.py:290-313) is downstream -- 11 affected dst rows of 512 leave 1 -
# (1 - 88/512)^8 = 78 % of the src rows (the CPU oracle on model_v2_lidar_b2_n4096)
ROWS_FLOOR_HEAD3 = 0.6

KNN_NAMES = ["src_knn_1", "src_knn_2", "src_knn_3", "dst_knn_1", "dst_knn_2", "dst_knn_3",
             "coarse_desc_knn", "coarse_nbr_src", "coarse_nbr_dst", "fine2_knn", "fine1_knn"]
PARTS = ("src", "dst")


def nerr(a, b):
    """max |a - b| / max |b| (0 for empty)"""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if b.size == 0:
        return 0.0
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def as_layout(r, B):
    """engine.hregnet_forward / oracle.hregnet_forward result -> fixture layout."""
    g = {}
    for part in PARTS:
        f = r[f"{part}_feats"]
        for lv in (1, 2, 3):
            for q in ("xyz", "sigmas", "desc"):
                g[f"{part}_{q}_{lv}"] = np.asarray(f[f"{q}_{lv}"])
            if "_fps_idx" in r:
                i = np.asarray(r["_fps_idx"][lv - 1])
                g[f"{part}_fps_{lv}"] = i[:B] if part == "src" else i[B:2 * B]
            else:
                g[f"{part}_fps_{lv}"] = np.asarray(f[f"fps_idx_{lv}"])
    for i, lv in enumerate((3, 2, 1)):
        g[f"R{lv}"] = np.asarray(r["rotation"][i])
        g[f"t{lv}"] = np.asarray(r["translation"][i])
        g[f"corres_{lv}"] = np.asarray(r[f"src_xyz_corres_{lv}"])
        if f"src_dst_weights_{lv}" in r:
            g[f"weights_{lv}"] = np.asarray(r[f"src_dst_weights_{lv}"])
    if "knn_sel" in r:  # oracle
        for k, v in r["knn_sel"].items():
            g["knn_" + k] = np.asarray(v)
    if "_knn" in r:  # engine.INDEX_RECORD (src and dst clouds stacked where both run)
        rec = {k: np.asarray(v) for k, v in r["_knn"].items()}
        for lv in (1, 2, 3):
            if f"knn_{lv}" in rec:
                g[f"knn_src_knn_{lv}"] = rec[f"knn_{lv}"][:B]
                g[f"knn_dst_knn_{lv}"] = rec[f"knn_{lv}"][B:2 * B]
        if "coarse_nbr" in rec:
            g["knn_coarse_nbr_src"] = rec["coarse_nbr"][:B]
            g["knn_coarse_nbr_dst"] = rec["coarse_nbr"][B:2 * B]
        for ours, name in (("coarse_desc_knn", "coarse_desc_knn"), ("fine_corres_2_knn", "fine2_knn"),
                           ("fine_corres_1_knn", "fine1_knn")):
            if ours in rec:
                g["knn_" + name] = rec[ours]
    return g


_SPREADS = None


def spread_table():
    """quantity ("xyz_3", "sigmas_2", "desc_1", "corres_3", "weights_2", ...) -> the largest
    normalised distance of the fp32 reference from its own float64 replay over the
    committed fixtures and both clouds.  Pooled over fixtures because a single tensor's
    distance is partly luck: on hregnet_lidar_b2_n4096 the reference's dst desc_3 sits
    6.7e-6 from float64 while the CPU oracle (numpy fp32) is 1.8e-5 and the layer-wise fp32
    GEMM path 1.5e-5 from it at the same, ill-conditioned element (tools/parity_probe.py)."""
    global _SPREADS
    if _SPREADS is None:
        from helpers import load_npz
        t = {}
        for name in SPREAD_FIXTURES:
            g = load_npz(name)
            for k in g:
                if not k.endswith("_64"):
                    continue
                base = k[:-3]
                q = base.replace("src_xyz_corres_", "corres_").replace("src_dst_weights_", "weights_")
                q = q[4:] if q.startswith(("src_", "dst_")) else q
                if q.startswith(("R", "t")) or base not in g or not q[-1].isdigit():
                    continue
                a, b = g[base], g[k]
                if q.startswith("desc_"):
                    a, b = a.transpose(0, 2, 1), b.transpose(0, 2, 1)
                t[q] = max(t.get(q, 0.0), nerr(a, b))
        _SPREADS = t
    return _SPREADS


def feat_bar(q):
    """bar for a quantity against float64: max(FEAT_TOL, SPREAD x the pooled reference
    spread); against a second fp32 result (no float64 twin), twice that"""
    return max(FEAT_TOL, SPREAD * spread_table().get(q, 0.0))


def _take(x, idx):
    """x [B,N,D], idx [B,...] -> [B,...,D]"""
    B = x.shape[0]
    flat = idx.reshape(B, -1).astype(np.int64)
    return np.take_along_axis(x, flat[..., None], 1).reshape(idx.shape + (x.shape[-1],))


def _same_point(a, b, tol=KP_TOL):
    return np.abs(a - b).max(-1) <= tol + tol * np.abs(b).max(-1)


def _transform(R, t, x):
    return np.einsum("bij,bnj->bni", R.astype(np.float64), x.astype(np.float64)) + t[:, None, :]


def _site_geometry(d, name):
    """(queries [B,M,D], database [B,N,D], database positions [B,N,3]) of a kNN site in
    layout d (the positions identify neighbours physically; for the 256-D descriptor kNN
    the database is the dst descriptors and the positions the dst level-3 keypoints)."""
    if name.endswith(("knn_1", "knn_2", "knn_3")) and name[:3] in PARTS:
        part, lv = name[:3], int(name[-1])
        db = d[part] if lv == 1 else d[f"{part}_xyz_{lv - 1}"]
        return _take(db, d[f"{part}_fps_{lv}"]), db, db
    if name == "coarse_desc_knn":
        return (d["src_desc_3"].transpose(0, 2, 1), d["dst_desc_3"].transpose(0, 2, 1),
                d["dst_xyz_3"])
    if name.startswith("coarse_nbr_"):
        x = d[f"{name[-3:]}_xyz_3"]
        return x, x, x
    if name == "fine2_knn":
        return _transform(d["R3"], d["t3"], d["src_xyz_2"]), d["dst_xyz_2"], d["dst_xyz_2"]
    if name == "fine1_knn":
        return _transform(d["R2"], d["t2"], d["src_xyz_1"]), d["dst_xyz_1"], d["dst_xyz_1"]
    raise KeyError(name)


def _knn_rows(ours, ref, name):
    """per query row: (mismatch of the selected neighbour SETS by position, float64
    boundary margin of the reference row, reference neighbour indices)"""
    _, _, pos_o = _site_geometry(ours, name)
    q_r, db_r, pos_r = _site_geometry(ref, name)
    io, ir = ours["knn_" + name], ref["knn_" + name]
    po, pr = _take(pos_o, io), _take(pos_r, ir)              # [B,M,k,3]
    close = _same_point(po[:, :, :, None, :], pr[:, :, None, :, :])  # [B,M,k,k]
    mism = ~(close.any(3).all(2) & close.any(2).all(2))
    margin = np.full(mism.shape, np.inf)
    k = ir.shape[-1]
    for b, m in zip(*np.nonzero(mism)):
        d = ((db_r[b].astype(np.float64) - q_r[b, m].astype(np.float64)) ** 2).sum(-1)
        ds = np.sort(d)
        if k < ds.size:
            margin[b, m] = (ds[k] - ds[k - 1]) / max(ds[k - 1], 1e-30)
    return mism, margin, ir


def _wfps_first_divergence(xyz, sigmas, idx_ours_in_ref, idx_ref):
    """(step, float64 relative margin) of a WFPS run's first divergence, replayed along
    the reference's selections on the reference's inputs (w = (1/(sigma+1e-5))/mean,
    models.py:30-32; d = w * |x - x_sel|^2, .cu:254-375); None if none."""
    diff = np.nonzero(idx_ours_in_ref != idx_ref)[0]
    if diff.size == 0:
        return None
    j = int(diff[0])
    x = xyz.astype(np.float64)
    w = 1.0 / (sigmas.astype(np.float64) + 1e-5)
    w = w / w.mean()
    temp = np.full(x.shape[0], 1e10)
    for t in range(j):
        temp = np.minimum(temp, w * ((x - x[idx_ref[t]]) ** 2).sum(-1))
    a, b = temp[idx_ref[j]], temp[idx_ours_in_ref[j]]
    return j, float((a - b) / max(abs(a), 1e-30))


def _root_cap(bad, label, n, rows):
    cap = max(ROOT_MIN, ROOT_FRAC * rows)
    if n > cap:
        bad.append(f"{label}: {n} root selection mismatches (near ties not downstream of "
                   f"another) > {cap:g}")


def _floor(bad, label, ok, floor=ROWS_FLOOR):
    n, tot = int(ok.sum()), int(ok.size)
    if tot and n < floor * tot:
        bad.append(f"{label}: only {n}/{tot} rows compared (< {floor:.0%}: too many rows "
                   "downstream of selection mismatches)")


def evaluate(ours, ref, continuous=True):
    """-> (stats dict, list of contract violations).  continuous=False: the selection
    contract, the row floor and R/t only (a reference without float64 twins of a different
    forward, e.g. the train-mode one)."""
    st, bad = {}, []
    B = ref["src"].shape[0]
    ours = {"src": ref["src"], "dst": ref["dst"], **ours}  # the same input clouds
    aff = {}  # (part, level) -> [B,M] bool: downstream of a selection mismatch

    def cont(key, label, ok, channel_major=False):
        """a continuous output on the rows `ok`: against the float64 replay when the
        reference has one (bar feat_bar), else against the fp32 result (bar 2 x feat_bar:
        each of two fp32 results within feat_bar of the exact values)"""
        if not continuous:
            return
        x, y = ours[key], ref[key]
        y64 = ref.get(key + "_64")
        if channel_major:
            x, y = x.transpose(0, 2, 1), y.transpose(0, 2, 1)
            y64 = None if y64 is None else y64.transpose(0, 2, 1)
        q = key[4:] if key.startswith(("src_", "dst_")) else key
        st[label + "_vs_ref32"] = nerr(x[ok], y[ok])
        if y64 is not None:
            e, bar = nerr(x[ok], y64[ok]), feat_bar(q)
            st[label + "_vs_f64"], st[label + "_ref32_vs_f64"] = e, nerr(y[ok], y64[ok])
        else:
            e, bar = st[label + "_vs_ref32"], 2 * feat_bar(q)
        st[label + "_bar"] = bar
        if e > bar:
            bad.append(f"{label}: {e:.2e} > bar {bar:.2e} on rows with identical selections")

    def knn_site(name, upstream_q, upstream_db):
        """kNN site: mismatched rows must be near ties unless their query / candidates
        are downstream of an earlier mismatch; returns the rows to mark affected."""
        if "knn_" + name not in ours or "knn_" + name not in ref:
            return None
        mism, margin, ir = _knn_rows(ours, ref, name)
        up = np.zeros(mism.shape, bool)
        if upstream_q is not None:
            up |= upstream_q
        if upstream_db is not None:
            up |= np.take_along_axis(upstream_db, ir.reshape(B, -1).astype(np.int64), 1
                                     ).reshape(ir.shape).any(-1)
        st[f"knn_{name}_mismatch"] = int(mism.sum())
        own = mism & ~up
        _root_cap(bad, f"kNN {name}", int(own.sum()), own.size)
        if own.any():
            mx = float(margin[own].max())
            st[f"knn_{name}_max_tie_margin"] = mx
            if mx > KNN_TIE:
                bad.append(f"kNN {name}: {int(own.sum())} rows differ, boundary margin {mx:.2e} > {KNN_TIE}")
        return mism | up

    for part in PARTS:
        for lv in (1, 2, 3):
            pre = f"{part}_L{lv}"
            M = ref[f"{part}_fps_{lv}"].shape[1]
            # selection of the level's centroids
            if lv == 1:
                sel_bad = ours[f"{part}_fps_1"] != ref[f"{part}_fps_1"]
                if sel_bad.any():
                    bad.append(f"{pre}: FPS indices differ ({int(sel_bad.sum())})")
                up_db = np.zeros((B, ref[part].shape[1]), bool)
            else:
                xo = _take(ours[f"{part}_xyz_{lv - 1}"], ours[f"{part}_fps_{lv}"])
                xr = _take(ref[f"{part}_xyz_{lv - 1}"], ref[f"{part}_fps_{lv}"])
                sel_bad = ~_same_point(xo, xr)
                up_db = aff[(part, lv - 1)]
                xref = ref[f"{part}_xyz_{lv - 1}"]
                roots = 0
                for c in np.nonzero(sel_bad.any(1))[0]:
                    d = ((xo[c][:, None, :].astype(np.float64) - xref[c][None]) ** 2).sum(-1)
                    dv = _wfps_first_divergence(xref[c], ref[f"{part}_sigmas_{lv - 1}"][c],
                                                d.argmin(1), ref[f"{part}_fps_{lv}"][c])
                    if dv is None:
                        continue
                    j, mg = dv
                    st[f"{pre}_wfps_cloud{c}_divergence"] = (j, mg)
                    if up_db[c].any():  # its weights / points moved upstream
                        continue
                    roots += 1
                    if abs(mg) > WFPS_TIE:
                        bad.append(f"{pre} cloud {c}: WFPS diverges at step {j}, margin {mg:.2e} > {WFPS_TIE}")
                st[f"{pre}_wfps_root_divergences"] = roots  # (at most one per cloud)
            st[f"{pre}_selection_mismatch"] = int(sel_bad.sum())
            a = knn_site(f"{part}_knn_{lv}", sel_bad, up_db)
            a = sel_bad if a is None else a
            aff[(part, lv)] = a
            ok = ~a
            st[f"{pre}_rows_compared"] = f"{int(ok.sum())}/{B * M}"
            _floor(bad, pre, ok)
            for q in ("xyz", "sigmas", "desc"):
                cont(f"{part}_{q}_{lv}", f"{pre}_{q}", ok, q == "desc")
    # CoarseReg (level 3): desc kNN src -> dst, neighbour branch xyz self-kNN on both clouds
    nbr = {}
    for part in PARTS:
        a = knn_site(f"coarse_nbr_{part}", aff[(part, 3)], aff[(part, 3)])
        nbr[part] = aff[(part, 3)] if a is None else a
    # a dst keypoint's neighbour-aware descriptor moves with any affected member of its group
    heads = {3: knn_site("coarse_desc_knn", nbr["src"], nbr["dst"]),
             2: knn_site("fine2_knn", aff[("src", 2)], aff[("dst", 2)]),
             1: knn_site("fine1_knn", aff[("src", 1)], aff[("dst", 1)])}
    for lv in (3, 2, 1):
        a = heads[lv] if heads[lv] is not None else aff[("src", lv)]
        ok = ~a
        for q in ("corres", "weights"):
            if f"{q}_{lv}" in ref:
                cont(f"{q}_{lv}", f"{q}_{lv}", ok)
        st[f"heads_L{lv}_rows_compared"] = f"{int(ok.sum())}/{ok.size}"
        _floor(bad, f"heads L{lv}", ok, ROWS_FLOOR_HEAD3 if lv == 3 else ROWS_FLOOR)
        st[f"_affected_heads_{lv}"] = a
        for q in ("R", "t"):
            e = float(np.abs(ours[f"{q}{lv}"] - ref[f"{q}{lv}"]).max())
            st[f"{q}{lv}_abs"] = e
            if e > RT_TOL:
                bad.append(f"{q}{lv}: {e:.2e} > {RT_TOL}")
    return st, bad


def report(st, title="", bad=None):
    lines = ["", "parity " + title]
    for k in sorted(st):
        if k.startswith("_"):
            continue
        v = st[k]
        if isinstance(v, float):
            v = "%.3e" % v
        elif isinstance(v, tuple):
            v = "step %d, margin %.3e" % v
        lines.append("  %-40s %s" % (k, v))
    lines.append("  %-40s %s" % ("RESULT", "FAIL: " + "; ".join(bad) if bad else "pass"))
    text = "\n".join(lines)
    print(text)
    path = os.environ.get("HREG_PARITY_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(text + "\n")


def check(ours, ref, title=""):
    """evaluate + print + assert; returns the stats"""
    st, bad = evaluate(ours, ref)
    report(st, title, bad)
    assert not bad, "\n".join(bad)
    return st
