"""Debug (CPU, needs /root/reference): the reference's fp64 training step on the fixture's
selections, with the level-3 DescExtractor inputs / output gradient and per-call
parameter gradients saved to tests/golden/_debug_l3.npz (not committed)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)
import make_golden as mg  # noqa: E402


def main():
    pu = mg.install_shims()
    sys.modules["pytorch3d.transforms"].matrix_to_euler_angles = mg.p3d_matrix_to_euler_angles
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_losses", os.path.join(mg.REF, "losses/losses.py"))
    L = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(L)
    from models.HRegNet.models import HRegNet
    from pcd_reg_hregnet_amd import weights
    fx = np.load(os.path.join(REPO, "tests/golden/train_step_b2_n2048.npz"))
    template = HRegNet(mg._Args()).state_dict()
    sd = weights.make_state_dict(template, seed=0, pretrained_feats=True)
    net = HRegNet(mg._Args())
    net.load_state_dict(sd)
    net = net.double().train()
    pu.replay = [torch.from_numpy(fx["idx_" + n]) for n in mg.TRAIN_FPS_NAMES]
    mg.KNN_REPLAY = [torch.from_numpy(fx["idx_" + n]).long() for n in mg.TRAIN_KNN_NAMES]
    caps = []
    m3 = net.feature_extraction.desc_extractor_3

    def hook(mod, inp, out):
        out.retain_grad()
        caps.append((inp[0].detach().clone(), inp[1].detach().clone(), out))

    h = m3.register_forward_hook(hook)
    te, tz = torch.eye, torch.zeros
    torch.eye = lambda *a, **k: te(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    torch.zeros = lambda *a, **k: tz(*a, **{**k, "dtype": k.get("dtype", torch.float64)})
    ret = net(torch.from_numpy(fx["src"]).double(), torch.from_numpy(fx["dst"]).double())
    gR, gt = torch.from_numpy(fx["R_gt"]).double(), torch.from_numpy(fx["t_gt"]).double()
    loss = 0.0
    for i in range(3):
        loss = loss + L.transformation_loss(ret["rotation"][i], ret["translation"][i], gR, gt, 1.0)[0]
    (loss / 3.0).backward()
    torch.eye, torch.zeros = te, tz
    h.remove()
    print("loss64", float(loss / 3.0), "fixture", float(fx["loss64"]))
    out = {}
    for ci, (g, am, d) in enumerate(caps):
        part = "src" if ci == 0 else "dst"
        out[f"{part}_grouped"] = g.numpy()
        out[f"{part}_att_map"] = am.numpy()
        out[f"{part}_d"] = d.detach().numpy()
        out[f"{part}_dgrad"] = d.grad.numpy()
        m3.zero_grad()
        x1 = m3.convs(g)
        x2 = torch.max(x1, dim=3, keepdim=True)[0].repeat(1, 1, 1, x1.shape[-1])
        y = torch.max(m3.mlp2(m3.mlp1(torch.cat((x2, x1, am), dim=1))), dim=3)[0]
        y.backward(d.grad)
        for n, p in m3.named_parameters():
            out[f"{part}_pgrad_{n}"] = p.grad.numpy().copy()
    np.savez(os.path.join(REPO, "tests/golden/_debug_l3.npz"), **out)
    print("written")


if __name__ == "__main__":
    main()
