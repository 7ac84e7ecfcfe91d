"""Time spatial_index_kernel variants (HREG_SI_EXP: 0 full, 1 no sort, 2 no boxes, 3 bbox+keys only).
usage: python tools/si_experiment.py  (GPU box; builds knn.hip variants into /tmp)"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tools.op_bench import timeit  # noqa: E402

SRC = os.path.join(REPO, "pcd_reg_hregnet_amd", "csrc", "knn.hip")


def main():
    torch.cuda.init()
    rng = np.random.default_rng(0)
    b, n = 16, 16384
    p = torch.from_numpy(rng.uniform(-40, 40, (b, n, 3)).astype(np.float32)).cuda()
    res = {}
    for exp in (0, 1, 2, 3):
        out = f"/tmp/si_{exp}.so"
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                               "-ffp-contract=off", "-shared", "-fPIC", f"-DHREG_SI_EXP={exp}", SRC,
                               "-o", out])
        L = ctypes.CDLL(out)
        L.hreg_spatial_index_bytes.restype = ctypes.c_size_t
        nbytes = L.hreg_spatial_index_bytes(b, n)
        ws = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        fn = lambda: L.hreg_spatial_index(ctypes.c_void_p(p.data_ptr()), b, n,  # noqa: E731
                                          ctypes.c_void_p(ws.data_ptr()), st)
        res[exp] = round(timeit(fn), 4)
    print(res)


if __name__ == "__main__":
    main()
