"""Calibration evaluation of the reference (metrics/calibeval.py) on the HIP library.

``CalibEval`` / ``MultiLayerCalibEval`` keep the reference's constructor, methods and
``results.json`` layout (calibeval.py:11-380; caller test/test_v3.py:100-140, one
evaluator per HRegNet level).  The per-pair work of ``add_batch`` -- the error
transform ``pred_tf @ gt_tf``, the XYZ Euler angles of the error and of the
prediction (pytorch3d's ``matrix_to_euler_angles``), the geodesic angle and the
translation norm with their batch means -- is one kernel (csrc/losses.hip
``calib_metrics_kernel``); the inputs stay on the GPU (the reference copies them to
the host first).  The accumulated lists and the mean / SD statistics are host
bookkeeping over a few numbers per pair, computed with numpy exactly as the reference
does -- including ``get_results``' unpacking of ``getSD()``, which swaps the rotation
and translation SDs in ``"sd"`` and ``"mean_sd"`` (calibeval.py:48-65 vs :140-165).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from . import _lib


def _tf(t: torch.Tensor, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"CalibEval: {name} must be a GPU tensor (no CPU fallback)")
    if t.dim() != 3 or tuple(t.shape[1:]) != (4, 4):
        raise ValueError(f"CalibEval: {name} has shape {tuple(t.shape)}, expected [B,4,4]")
    return t.detach().float().contiguous()


def calib_metrics(gt_tf: torch.Tensor, pred_tf: torch.Tensor):
    """-> (per_pair [B][12] on the GPU, batch geodesic [2] on the GPU); see module doc."""
    g = _tf(gt_tf, "gt_tf")
    p = _tf(pred_tf, "pred_tf")
    B = p.shape[0]
    if B == 0 or g.shape[0] != B:
        raise ValueError("CalibEval: empty batch or batch sizes differ")
    per = torch.empty(B, 12, device=p.device)
    geo = torch.empty(2, device=p.device)
    _lib.call("hreg_calib_metrics", p, g, B, per, geo, _lib.stream_handle())
    return per, geo


class CalibEval:
    """metrics/calibeval.py:11-330."""

    def __init__(self, config=None, translation_threshold=None, rotation_threshold=None):
        self.config = config
        self.translation_threshold = translation_threshold
        self.rotation_threshold = rotation_threshold
        self.reset()

    def reset(self) -> None:
        self.loss_r = []
        self.loss_t = []
        self.geodesic = []
        self.success_idx = []
        self.pred = []
        self.results = {}

    def add_batch(self, gt_tf, pred_tf, idx=None, return_results=False) -> None:
        per, geo = calib_metrics(gt_tf, pred_tf)
        self.add_computed(per.cpu().numpy(), geo.cpu().numpy())

    def add_computed(self, per_pair: np.ndarray, batch_geo: np.ndarray) -> None:
        """Append one batch's kernel outputs (per_pair [B][12], batch_geo [2]) to the
        lists, as float32 values like the reference's ``.tolist()`` of fp32 tensors."""
        per = np.asarray(per_pair, dtype=np.float32)
        self.loss_r.extend(per[:, 0:3].tolist())
        self.loss_t.extend(per[:, 3:6].tolist())
        self.pred.extend(per[:, 6:12].tolist())
        self.geodesic.append([float(v) for v in np.asarray(batch_geo, dtype=np.float32)])

    def get_stats(self):
        if self.success_idx:
            sel = np.asarray(self.success_idx)
            loss_r = np.abs(np.asarray(self.loss_r)[sel]).mean(axis=0)
            loss_t = np.abs(np.asarray(self.loss_t)[sel]).mean(axis=0)
            geodesic = np.asarray(self.geodesic)[sel].mean(axis=0)
        else:
            loss_r = np.abs(np.asarray(self.loss_r)).mean(axis=0)
            loss_t = np.abs(np.asarray(self.loss_t)).mean(axis=0)
            geodesic = np.asarray(self.geodesic).mean(axis=0)
        return loss_r, loss_t, geodesic

    def getSD(self):
        geo = np.asarray(self.geodesic)
        if self.success_idx:
            sel = np.asarray(self.success_idx)
            loss_r = np.abs(np.asarray(self.loss_r)[sel]).std(axis=0)
            loss_t = np.abs(np.asarray(self.loss_t)[sel]).std(axis=0)
            sd_dR = np.abs(geo[sel, 0]).std(axis=0)
            sd_dT = np.abs(geo[sel, 1]).std(axis=0)
        else:
            loss_r = np.abs(np.asarray(self.loss_r)).std(axis=0)
            loss_t = np.abs(np.asarray(self.loss_t)).std(axis=0)
            sd_dR = np.abs(geo[:, 0]).std(axis=0)
            sd_dT = np.abs(geo[:, 1]).std(axis=0)
        return loss_r, loss_t, sd_dR, sd_dT

    def compute_recall(self) -> float:
        return len(self.success_idx) / len(self.loss_r) if self.loss_r else 0.0

    def get_results(self) -> dict:
        r, t, g = self.get_stats()
        sd_t, sd_r, sd_dR, sd_dT = self.getSD()  # (sic) calibeval.py:48: names swapped
        self.results = {
            "pred_calib": self.pred,
            "error_calib": np.concatenate((self.loss_r, self.loss_t), axis=1).tolist(),
            "mean_error": sum([r.tolist(), t.tolist(), g.tolist()], []),
            "sd": sum([sd_r.tolist(), sd_t.tolist()], []),
            "mean_sd": [np.mean(sd_r).tolist(), np.mean(sd_t).tolist()],
            "mean_sd_dRT": [np.mean(sd_dR).tolist(), np.mean(sd_dT).tolist()],
        }
        return self.results

    def geodesic_distance(self, x: torch.Tensor) -> list:
        """calibeval.py:197-214 on an error transform [B,4,4] -> [mean deg, mean norm]."""
        eye = torch.eye(4, device=x.device).expand(x.shape[0], 4, 4)
        _, geo = calib_metrics(eye, x)
        return [float(v) for v in geo.cpu().tolist()]

    @staticmethod
    def rotation_matrix_to_euler(rotation_matrix: torch.Tensor) -> torch.Tensor:
        """calibeval.py:217-225: XYZ Euler angles in degrees, [B,3,3] -> [B,3]."""
        B = rotation_matrix.shape[0]
        tf = torch.eye(4, device=rotation_matrix.device).repeat(B, 1, 1)
        tf[:, :3, :3] = rotation_matrix
        per, _ = calib_metrics(torch.eye(4, device=tf.device).expand(B, 4, 4), tf)
        return per[:, 6:9]

    @staticmethod
    def get_rotation_translation_from_transform(tf):
        return tf[..., :3, :3], tf[..., :3, 3]

    @staticmethod
    def compute_norm(tensor_a, tensor_b):
        assert tensor_a.shape == tensor_b.shape, "Shapes of input tensors must be the same"
        return tensor_a - tensor_b

    @staticmethod
    def relative_rotation_error(gt_rotations, rotations):
        """calibeval.py:258-276 (degrees), on the transformation-loss kernel's geodesic."""
        from .losses import calc_rot_rre_err
        return calc_rot_rre_err(rotations, gt_rotations)[1]

    def save_results(self) -> None:
        """calibeval.py:279-334: results.json under config.dataset_config.results_path."""
        self.get_results()
        dc = self.config.dataset_config
        name = ("results_" + "_" + self.config.dataset + "_" + dc.distribution + "_" +
                str(dc.max_rot_error) + "_" + str(dc.max_trans_error) + ".json")
        with open(os.path.join(dc.results_path, name), "w") as f:
            json.dump(self.results, f, indent=4)


class MultiLayerCalibEval:
    """metrics/calibeval.py:340-380: one CalibEval per level, combined results.json."""

    def __init__(self, config, num_layers=3, translation_threshold=None, rotation_threshold=None):
        self.config = config
        self.num_layers = num_layers
        self.evaluators = {layer: CalibEval(config, translation_threshold, rotation_threshold)
                           for layer in range(num_layers)}

    def reset(self):
        for ev in self.evaluators.values():
            ev.reset()

    def add_batch(self, layer, gt_tf, pred_tf, idx=None, return_results=False):
        if layer not in self.evaluators:
            raise ValueError(f"Layer {layer} is not valid. Valid layers: 0 to {self.num_layers - 1}.")
        self.evaluators[layer].add_batch(gt_tf, pred_tf, idx, return_results)

    def all_results(self) -> dict:
        combined = {f"layer_{layer}": ev.get_results() for layer, ev in self.evaluators.items()}
        dc = self.config.dataset_config
        combined.update({"dataset": self.config.dataset + dc.version, "model": dc.model,
                         "translation": dc.max_trans_error, "rotation": dc.max_rot_error,
                         "distribution": dc.distribution})
        return combined

    def save_all_results(self, output_file):
        with open(output_file, "w") as f:
            json.dump(self.all_results(), f, indent=4)


def pred_tf(R: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """test/test_v3.py:50-69 get_pred_tf: [B,3,3], [B,3] -> [B,4,4]."""
    B = R.shape[0]
    tf = torch.eye(4, device=R.device).repeat(B, 1, 1)
    tf[:, :3, :3] = R
    tf[:, :3, 3] = t
    return tf
