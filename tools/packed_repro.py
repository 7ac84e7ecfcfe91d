"""Does the packed-fp32 defect of DESIGN.md 4b still reproduce?  Run under a library built
with packed fp32 VALU ops in the bf16x6 kernels (tools/build_variant.py ... --packed,
selected by HREG_LIB) and under the product build: the eager forward at configs[1]
(B = 8, 2 x 16384 points) repeated, each repeat bitwise against the first, and a digest of
every output so the two builds can be compared bitwise.

  HREG_LIB=tools/b6exp_allpacked.so python tools/packed_repro.py; python tools/packed_repro.py
"""
import hashlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    from helpers import Args, state_dict_torch
    from pcd_reg_hregnet_amd import _lib, engine, synthetic
    from pcd_reg_hregnet_amd.models import HRegNet
    _lib.load()
    print("library:", _lib.LIB_PATH)
    net = HRegNet(Args())
    net.load_state_dict(state_dict_torch())
    P = net.cuda().eval().prepared(torch.device("cuda"))
    s, d, _, _ = synthetic.lidar_batch(8, 16384, seed0=100)
    src, dst = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()

    def digest():
        with torch.no_grad():
            r = engine.hregnet_forward(P, src, dst)
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for part in ("src_feats", "dst_feats"):
            for k in sorted(r[part]):
                h.update(r[part][k].contiguous().cpu().numpy().tobytes())
        for x in r["rotation"] + r["translation"]:
            h.update(x.cpu().numpy().tobytes())
        return h.hexdigest()[:16]

    first = digest()
    reps = [digest() for _ in range(8)]
    print("forward digest", first, "repeats identical:", all(x == first for x in reps))


if __name__ == "__main__":
    main()
