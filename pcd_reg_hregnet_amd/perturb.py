"""Data side in front of the path: decalibration perturbations.

The reference builds each training pair in a DataLoader worker on the CPU:
``TruckScenesPerturbation.lidar_to_lidar`` (dataset/man_dataset.py:606-631) draws a
twist with ``UniformTransformSE3`` (transform/dataset_transforms.py:65-145), maps it
through the SE(3) exponential (transform/rodrigues.py:526-553) and moves the
calibrated cloud by it; the training loop then inverts ``igt``
(train/train_reg_v0.py:268-271).  Clouds were range-filtered and resampled before
that (dataset/dataset_utils.py:113-127, 177-223).

Here the random draws stay on the host generators the reference uses (torch's CPU
generator for the twists, numpy's global RandomState for the resampler), so a
seeded run draws the same numbers; all per-point and per-transform arithmetic runs
on the GPU through the C ABI (csrc/perturb.hip), batched over clouds:

* ``SO3`` / ``SE3``: exp / log / inverse / transform with the reference's names.
* ``UniformTransformSE3``: same constructor and ``generate_transform`` /
  ``apply_transform`` / ``__call__``; ``generate_transforms(n)`` draws n twists in
  one launch, equal to n consecutive ``generate_transform`` calls.
* ``create_perturb_file`` / ``load_perturb_file``: the ``perturbations_file_<split>.txt``
  CSV of 6-vectors (man_dataset.py:500-545).
* ``PerturbationPipeline``: ``lidar_to_lidar`` over a batch [B, N, 3] on the GPU ->
  ``uncalibed_pcd``, ``igt`` and the loop's ``gt = inverse(igt)``.
* ``PointCloudFilter`` (range filter, order-preserving GPU compaction) and
  ``PointCloudResampler`` (numpy's ``np.random.choice`` draws, GPU gather).

There is no CPU fallback: every op raises without the HIP library and a GPU.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from ._lib import call

_DIST = {"uniform": _lib.HREG_TWIST_UNIFORM, "gaussian": _lib.HREG_TWIST_GAUSSIAN,
         "inverse_gaussian": _lib.HREG_TWIST_INVERSE_GAUSSIAN}


def _stream():
    return _lib.stream_handle()


def _dev(t: torch.Tensor) -> torch.Tensor:
    if not t.is_cuda:
        raise RuntimeError("pcd_reg_hregnet_amd.perturb: tensors must be on the GPU "
                           "(there is no CPU fallback)")
    return t.contiguous().float()


class SO3:
    """transform/rodrigues.py:249-398 (the parts the data pipeline uses)."""

    @staticmethod
    def exp(w: torch.Tensor) -> torch.Tensor:
        """[*, 3] -> [*, 3, 3] (rodrigues.py:304-314)."""
        x = torch.cat([w.reshape(-1, 3), torch.zeros_like(w.reshape(-1, 3))], 1)
        return SE3.exp(x)[:, :3, :3].reshape(*w.shape[:-1], 3, 3)

    @staticmethod
    def log(R: torch.Tensor) -> torch.Tensor:
        """[*, 3, 3] -> [*, 3] (rodrigues.py:330-370)."""
        g = torch.zeros(*R.shape[:-2], 4, 4, device=R.device)
        g[..., :3, :3] = R
        g[..., 3, 3] = 1
        return SE3.log(g)[..., :3]

    @staticmethod
    def inverse(R: torch.Tensor) -> torch.Tensor:
        return R.transpose(-1, -2)


class SE3:
    """transform/rodrigues.py:470-617 on the GPU: twists [*, 6] <-> [*, 4, 4]."""

    @staticmethod
    def exp(x: torch.Tensor) -> torch.Tensor:
        x_ = _dev(x).reshape(-1, 6)
        g = torch.empty(x_.shape[0], 4, 4, device=x_.device)
        call("hreg_se3_exp", x_, x_.shape[0], g, _stream())
        return g.reshape(*x.shape[:-1], 4, 4)

    @staticmethod
    def log(g: torch.Tensor) -> torch.Tensor:
        g_ = _dev(g).reshape(-1, 4, 4)
        x = torch.empty(g_.shape[0], 6, device=g_.device)
        call("hreg_se3_log", g_, g_.shape[0], x, _stream())
        return x.reshape(*g.shape[:-2], 6)

    @staticmethod
    def inverse(g: torch.Tensor) -> torch.Tensor:
        """[R p; 0 1]^-1 = [R^T -R^T p; 0 1] (rodrigues.py:556-568)."""
        R = g[..., :3, :3]
        p = g[..., :3, 3:]
        out = torch.zeros_like(g)
        out[..., :3, :3] = R.transpose(-1, -2)
        out[..., :3, 3:] = -(R.transpose(-1, -2) @ p)
        out[..., 3, 3] = 1
        return out

    @staticmethod
    def transform(g: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
        """g [B, 4, 4], a [B, 3, N] -> R a + p (rodrigues.py:585-596), through the
        point-transform kernel (points as rows)."""
        B = g.shape[0]
        pts = _dev(a.transpose(-1, -2))
        out = torch.empty_like(pts)
        R = _dev(g[:, :3, :3])
        t = _dev(g[:, :3, 3])
        call("hreg_transform_points", pts, R, t, B, pts.shape[1], out, _stream())
        return out.transpose(-1, -2)


def _draws(n: int, randomly: bool, distribution: str):
    """The random numbers n consecutive generate_transform() calls consume, in the
    reference's order (dataset_transforms.py:80-122): (deg, tran) magnitudes when
    mag_randomly, then the w and t draws."""
    mags = np.empty((n, 2))
    s = np.empty((n, 6), np.float32)
    if distribution == "uniform":
        k = 8 if randomly else 6
        u = torch.rand(n * k).view(n, k)  # one bulk draw == the sequence of small draws
        if randomly:
            mags[:] = u[:, :2].double().numpy()
        s[:] = u[:, k - 6:].numpy()
    else:
        from scipy.stats import invgauss
        for i in range(n):
            if randomly:
                mags[i, 0] = torch.rand(1).item()
                mags[i, 1] = torch.rand(1).item()
            if distribution == "gaussian":
                s[i, :3] = torch.randn(1, 3).numpy()
                s[i, 3:] = torch.randn(1, 3).numpy()
            else:
                s[i, :3] = invgauss.rvs(mu=1.0, scale=0.1, size=3)
                s[i, 3:] = invgauss.rvs(mu=0.01, scale=0.002, size=3)
    return mags, s


class UniformTransformSE3:
    """transform/dataset_transforms.py:65-145 (same constructor, same draws)."""

    def __init__(self, max_deg, max_tran, distribution="uniform", mag_randomly=False,
                 concat=False, device=None):
        if distribution not in _DIST:
            raise NameError("Invalid distribution %s" % distribution)
        self.max_deg = max_deg
        self.max_tran = max_tran
        self.randomly = mag_randomly
        self.concat = concat
        self.distribution = distribution
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.gt = None
        self.igt = None

    def generate_transforms(self, n: int) -> torch.Tensor:
        """n twists [n, 6] on the GPU, equal to n consecutive generate_transform()."""
        mags, s = _draws(n, self.randomly, self.distribution)
        amp_tran = np.empty((n, 2), np.float32)
        for i in range(n):
            # python-float magnitudes, rounded to float32 where they scale a tensor
            deg = mags[i, 0] * self.max_deg if self.randomly else self.max_deg
            tran = mags[i, 1] * self.max_tran if self.randomly else self.max_tran
            amp_tran[i] = (deg * math.pi / 180.0, tran)
        sd = torch.from_numpy(s).to(self.device)
        at = torch.from_numpy(amp_tran).to(self.device)
        x = torch.empty(n, 6, device=self.device)
        call("hreg_twists_from_samples", sd, at, n, _DIST[self.distribution], x, _stream())
        return x

    def generate_transform(self) -> torch.Tensor:
        return self.generate_transforms(1)  # [1, 6]

    def apply_transform(self, p0: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        """p0 [1, 3, N] or [3, N] ([.., 6, N] with concat: xyz moved, normals rotated),
        x [1, 6] -> moved cloud of p0's shape; sets gt / igt (dataset_transforms.py:128-141)."""
        g = SE3.exp(x)
        self.gt = SE3.exp(-x).squeeze(0)
        self.igt = g.squeeze(0)
        p = p0.reshape(-1, p0.shape[-1])
        moved = SE3.transform(g, p[None, :3])[0]
        if self.concat:
            rot = SE3.transform(torch.cat([g[:, :, :3], torch.zeros_like(g[:, :, 3:])], 2),
                                p[None, 3:])[0]
            moved = torch.cat([moved, rot], 0)
        return moved.reshape(p0.shape)

    def transform(self, tensor):
        return self.apply_transform(tensor, self.generate_transform())

    def __call__(self, tensor):
        return self.transform(tensor)


def create_perturb_file(path: str, length: int, transform: UniformTransformSE3) -> None:
    """man_dataset.py:528-545: `length` twists, one per line, comma separated."""
    x = transform.generate_transforms(length).double().cpu().numpy()
    np.savetxt(path, x, delimiter=",")


def load_perturb_file(path: str) -> np.ndarray:
    """man_dataset.py:500-507: float32 [length, 6]."""
    return np.loadtxt(path, dtype=np.float32, delimiter=",").reshape(-1, 6)


class PerturbationPipeline:
    """TruckScenesPerturbation in L2L mode (man_dataset.py:476-631), batched on the GPU.

    split 'train': fresh twists from UniformTransformSE3 per cloud; other splits: the
    twists of the perturbation file (created on first use, as the reference does)."""

    def __init__(self, split="train", max_rot_error=20.0, max_trans_error=0.5,
                 mag_randomly=True, distribution="uniform", perturbations_file=None,
                 dataset_len=None, device=None):
        self.split = split
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self.transform = UniformTransformSE3(max_rot_error, max_trans_error, distribution,
                                             mag_randomly, device=self.device)
        self.perturb = None
        if split != "train" and perturbations_file:
            import os
            path = perturbations_file + split + ".txt"
            if not os.path.exists(path):
                if dataset_len is None:
                    raise ValueError("creating a perturbation file needs dataset_len")
                create_perturb_file(path, dataset_len, self.transform)
            self.perturb = torch.from_numpy(load_perturb_file(path)).to(self.device)

    def lidar_to_lidar(self, pcd_right: torch.Tensor, indices=None) -> dict:
        """pcd_right [B, N, 3] (calibrated) -> {uncalibed_pcd [B, N, 3], igt [B, 4, 4],
        gt [B, 4, 4] = igt^-1}; indices pick the file's twists outside 'train'."""
        pts = _dev(pcd_right)
        B, N, _ = pts.shape
        if self.perturb is not None:
            if indices is None:
                raise ValueError("lidar_to_lidar outside 'train' needs the sample indices")
            x = self.perturb[torch.as_tensor(indices, device=self.device).long()].contiguous()
        else:
            x = self.transform.generate_transforms(B)
        out = torch.empty_like(pts)
        igt = torch.empty(B, 4, 4, device=pts.device)
        gt = torch.empty(B, 4, 4, device=pts.device)
        call("hreg_perturb_clouds", pts, x, B, N, out, igt, gt, _stream())
        return {"uncalibed_pcd": out, "igt": igt, "gt": gt, "twist": x}


class PointCloudFilter:
    """dataset_utils.py:99-127 (the range filter; voxel down-sampling needs open3d and
    is not on the reference's L2L path, man_dataset.py:383-384)."""

    def __init__(self, max_range: float = 100.0):
        self._max_range = max_range

    def remove_points_by_range(self, point_cloud: torch.Tensor, intensity=None):
        """[B, N, 3] (or [N, 3]) -> (packed points, packed intensity or None, counts [B]):
        row b holds its counts[b] kept points first, in input order."""
        single = point_cloud.dim() == 2
        pts = _dev(point_cloud[None] if single else point_cloud)
        B, N, _ = pts.shape
        inten = None if intensity is None else _dev(intensity.reshape(B, N))
        out = torch.zeros_like(pts)
        oint = None if inten is None else torch.zeros_like(inten)
        counts = torch.empty(B, dtype=torch.int32, device=pts.device)
        call("hreg_range_filter", pts, inten, B, N, float(self._max_range), out, oint, counts,
             _stream())
        if single:
            n = int(counts[0])
            return out[0, :n], (None if oint is None else oint[0, :n]), counts
        return out, oint, counts

    def __call__(self, point_cloud, intensity=None):
        return self.remove_points_by_range(point_cloud, intensity)


class PointCloudResampler:
    """dataset_utils.py:177-223: pad with np.random.choice(n, pad, replace=True) copies
    or subsample np.random.choice(n, num_points, replace=False) -- numpy's global
    RandomState draws the indices exactly as the reference does; the rows are
    gathered on the GPU."""

    def __init__(self, num_points: int = 1024):
        self._num_points = num_points

    def indices(self, n: int) -> np.ndarray:
        if self._num_points == -1:
            return np.arange(n)
        if n <= self._num_points:
            pad = np.random.choice(n, self._num_points - n, replace=True)
            return np.concatenate([np.arange(n), pad])
        return np.random.choice(n, self._num_points, replace=False)

    def __call__(self, point_cloud: torch.Tensor, intensity=None):
        pts = _dev(point_cloud)
        n = pts.shape[0]
        idx = torch.from_numpy(self.indices(n).astype(np.int32)).to(pts.device)
        M = idx.shape[0]
        out = torch.empty(M, 3, device=pts.device)
        call("hreg_gather_rows", pts, 3, idx, M, 3, out, 3, _stream())
        if intensity is None:
            return out, None
        inten = _dev(intensity).reshape(n, 1)
        oi = torch.empty(M, 1, device=pts.device)
        call("hreg_gather_rows", inten, 1, idx, M, 1, oi, 1, _stream())
        return out, oi.reshape(M)
