"""Debug: is the level-3 DescExtractor backward of the training graph locally right?

Runs the fixture training step with the reference selections, captures the level-3
grouped rows / attentive map / descriptor (and its gradient) of both calls, replays the
DescExtractor in float64 torch on those tensors with the captured descriptor gradient
and compares its parameter gradients with ours."""
import copy
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from pcd_reg_hregnet_amd import engine, train_graph as tgm  # noqa: E402

CAP = []
FEAT_KEYS = ["xyz_1", "xyz_2", "xyz_3", "sigmas_1", "sigmas_2", "sigmas_3", "desc_1", "desc_2",
             "desc_3"]
orig_group_max = tgm.group_max
orig_cat_rows = tgm.cat_rows


def desc_fwd(m, g, am):
    """DescExtractor.forward (reference layers.py:200-209) on the module's layers."""
    x1 = m.convs(g)
    x2 = torch.max(x1, dim=3, keepdim=True)[0].repeat(1, 1, 1, x1.shape[-1])
    x2 = torch.cat((x2, x1, am), dim=1)
    return torch.max(m.mlp2(m.mlp1(x2)), dim=3)[0]


def main():
    from helpers import Args, load_npz, state_dict_torch
    from pcd_reg_hregnet_amd.models import HRegNet
    fx = load_npz("train_step_b2_n2048.npz")
    net = HRegNet(Args())
    net.load_state_dict(state_dict_torch())
    net = net.cuda().train()
    net_ref = copy.deepcopy(net).double()
    # capture inputs of each desc extractor call by wrapping seq_convs on desc.convs
    orig_kl = tgm.keypoint_level

    def kl(det, desc, lvl, xyz, feats, weights, hook=None, part="src"):
        rec = {"lvl": lvl, "part": part}
        o_seq = tgm.seq_convs

        def seq(x, s):
            if s is desc.convs:
                rec["grouped"] = x.detach().clone()
            return o_seq(x, s)

        o_cat = tgm.cat_rows

        def cat(*blocks):
            if len(blocks) == 3 and isinstance(blocks[0], tuple):
                rec["att_map"] = blocks[2].detach().clone()
            return o_cat(*blocks)

        tgm.seq_convs, tgm.cat_rows = seq, cat
        try:
            out = orig_kl(det, desc, lvl, xyz, feats, weights, hook, part)
        finally:
            tgm.seq_convs, tgm.cat_rows = o_seq, o_cat
        d = out[3]
        d.retain_grad()
        rec["d"] = d
        CAP.append(rec)
        return out

    tgm.keypoint_level = kl
    FE = {}
    orig_fe = tgm.feature_extraction

    def fe(f, points, hook=None, part="src"):
        out = orig_fe(f, points, hook, part)
        for kk in FEAT_KEYS:
            out[kk].retain_grad()
        FE[part] = out
        return out

    tgm.feature_extraction = fe
    inject = {k[4:]: fx[k] for k in fx if k.startswith("idx_")}
    hook = tgm.IndexHook(inject)
    ret = tgm.hregnet_train_forward(net, torch.from_numpy(fx["src"]).cuda(),
                                    torch.from_numpy(fx["dst"]).cuda(), hook)
    loss, _, _ = tgm.registration_loss(ret, torch.from_numpy(fx["R_gt"]).cuda(),
                                       torch.from_numpy(fx["t_gt"]).cuda())
    loss.backward()
    torch.cuda.synchronize()
    print("loss", float(loss), "ref", float(fx["loss"]))
    for part in ("src", "dst"):
        for kk in FEAT_KEYS:
            t = FE[part][kk]
            g = t.grad.double().cpu().numpy()
            v = t.detach().double().cpu().numpy()
            r32 = fx[f"fgrad_{part}_{kk}"].astype(np.float64)
            r64 = fx[f"fgrad_{part}_{kk}_64"]
            if kk.startswith("desc"):
                g = g.reshape(r64.shape[0], r64.shape[2], r64.shape[1]).transpose(0, 2, 1)
                v = v.reshape(r64.shape[0], r64.shape[2], r64.shape[1]).transpose(0, 2, 1)
            g = g.reshape(r64.shape)
            v = v.reshape(r64.shape)
            vref = fx[f"feat_{part}_{kk}_64"]
            e_o = np.linalg.norm(g - r64) / np.linalg.norm(r64)
            e_r = np.linalg.norm(r32 - r64) / np.linalg.norm(r64)
            dv = np.abs(v - vref).max()
            print(f"{part} {kk:9s} grad rel err ours {e_o:.2e}  fp32 ref {e_r:.2e}   value max|d| {dv:.2e}")
            if e_o > 10 * e_r and kk.startswith("desc"):
                diff = np.abs(g - r64)
                # where the error sits: per point (max over channels)
                per_pt = diff.max(axis=1)
                idx = np.argsort(per_pt.reshape(-1))[::-1][:8]
                print("   worst points (b*M+m, max err, grad scale at point):",
                      [(int(i), float(per_pt.reshape(-1)[i]),
                        float(np.abs(r64.transpose(0, 2, 1).reshape(-1, r64.shape[1])[i]).max()))
                       for i in idx])
    dbg = np.load(os.path.join(REPO, "tests/golden/_debug_l3.npz"))
    M, k = engine.LEVELS[2][:2]
    m3 = net_ref.feature_extraction.desc_extractor_3
    for rec in CAP:
        if rec["lvl"] != 2:
            continue
        part = rec["part"]
        nb = rec["grouped"].shape[0] // (M * k)
        g = rec["grouped"].double().view(nb, M, k, -1).permute(0, 3, 1, 2).contiguous()
        am = rec["att_map"].double().view(nb, M, k, -1).permute(0, 3, 1, 2).contiguous()
        gd = rec["d"].grad.double().view(nb, M, -1).permute(0, 2, 1).contiguous()
        rg = torch.from_numpy(dbg[f"{part}_grouped"]).cuda()
        ram = torch.from_numpy(dbg[f"{part}_att_map"]).cuda()
        rgd = torch.from_numpy(dbg[f"{part}_dgrad"]).cuda()
        for nm, a, b in (("grouped", g, rg), ("att_map", am, ram), ("dgrad", gd, rgd)):
            e = (a - b).abs()
            print(f"L3 {part} {nm}: max|d| {float(e.max()):.3e} scale {float(b.abs().max()):.3e}"
                  f" rel-norm {float((a - b).norm() / b.norm()):.3e}")
            if nm != "dgrad":
                per_c = e.amax(dim=(0, 2, 3))
                top = torch.argsort(per_c, descending=True)[:6]
                print("     worst channels:", [(int(c), float(per_c[c])) for c in top])
        with torch.no_grad():
            def parts(gi, ai):
                x1 = m3.convs(gi)
                x2 = torch.max(x1, dim=3, keepdim=True)[0].repeat(1, 1, 1, x1.shape[-1])
                y1 = m3.mlp1(torch.cat((x2, x1, ai), dim=1))
                y2 = m3.mlp2(y1)
                return x1, y1, y2
            A = parts(g, am)
            Bp = parts(rg, ram)
            for nm, a, b in (("x1 kmax", A[0], Bp[0]), ("y2 kmax", A[2], Bp[2])):
                ia, ib = a.argmax(dim=3), b.argmax(dim=3)
                flips = (ia != ib).nonzero()
                srt = torch.sort(b, dim=3, descending=True)[0]
                print(f"   {nm}: {flips.shape[0]} argmax flips; ", [
                    (tuple(int(v) for v in f), float(srt[tuple(f)][0] - srt[tuple(f)][1]))
                    for f in flips[:5]])
            for nm, a, b in (("x1 relu", A[0], Bp[0]), ("y1 relu", A[1], Bp[1])):
                print(f"   {nm}: {int(((a > 0) != (b > 0)).sum())} relu flips")
        for label, gi, ai, di in (("ref-in ours-dgrad", rg, ram, gd), ("ours-in ref-dgrad", g, am, rgd),
                                  ("ref-in ref-dgrad", rg, ram, rgd)):
            m3.zero_grad()
            y = desc_fwd(m3, gi, ai)
            y.backward(di)
            p = dict(m3.named_parameters())["mlp1.1.bias"].grad
            r = torch.from_numpy(dbg[f"{part}_pgrad_mlp1.1.bias"]).cuda()
            print(f"  {part} {label}: mlp1.1.bias rel err {float((p - r).norm() / r.norm()):.3e}")
    for lvl in (0, 1, 2):
        name = f"desc_extractor_{lvl + 1}"
        M, k = engine.LEVELS[lvl][:2]
        ref_mod = getattr(net_ref.feature_extraction, name)
        ref_mod.zero_grad()
        for rec in CAP:
            if rec["lvl"] != lvl:
                continue
            g = rec["grouped"].double()
            nb = g.shape[0] // (M * k)
            gin = g.view(nb, M, k, -1).permute(0, 3, 1, 2).contiguous()
            am = rec["att_map"].double().view(nb, M, k, -1).permute(0, 3, 1, 2).contiguous()
            d_ref = desc_fwd(ref_mod, gin, am)  # [nb, Cd, M]
            d_ours = rec["d"].detach().double().view(nb, M, -1).permute(0, 2, 1)
            print(f"L{lvl + 1} {rec['part']} desc fwd max|diff| {float((d_ref - d_ours).abs().max()):.3e}"
                  f" scale {float(d_ref.abs().max()):.3e}")
            gd = rec["d"].grad.double().view(nb, M, -1).permute(0, 2, 1)
            d_ref.backward(gd)
        ours = dict(getattr(net.feature_extraction, name).named_parameters())
        for pn, p in ref_mod.named_parameters():
            a = ours[pn].grad.double().cpu()
            b = p.grad.cpu()
            err = float((a - b).norm() / max(float(b.norm()), 1e-30))
            print(f"  {name}.{pn:18s} rel err (ours vs fp64 replay on our inputs) {err:.3e}"
                  f"  |g| {float(b.norm()):.3e}")


if __name__ == "__main__":
    main()
