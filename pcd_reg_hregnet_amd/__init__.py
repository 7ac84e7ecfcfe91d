"""MI355X-native HRegNet registration forward (gfx950 HIP kernels behind a C ABI).

Drop-in surface of the reference (UpendraArun/pcd_reg_hregnet):
  HRegNet, HierFeatureExtraction           (models/HRegNet/models.py)
  Model_V2                                 (models/model_v2/models.py, inference)
  furthest_point_sample, weighted_furthest_point_sample, gather_operation, set_seed
                                           (models/utils.py)
  point_utils_cuda                          (models/PointUtils, pybind module)
  knn_points, knn_gather                    (pytorch3d.ops as HRegNet calls it)
  transformation_loss, calc_rot_rre_err, calc_tran_rte_err   (losses/losses.py)
"""
from .models import HRegNet, HierFeatureExtraction, Model_V2  # noqa: F401
from .utils import (furthest_point_sample, weighted_furthest_point_sample,  # noqa: F401
                    gather_operation, set_seed, calc_error_np)
from .knn import knn_points, knn_gather  # noqa: F401
from .losses import transformation_loss, calc_rot_rre_err, calc_tran_rte_err  # noqa: F401
from . import point_utils_cuda  # noqa: F401
from . import train as _train, trainer as _trainer, switches as _switches  # noqa: F401

_switches.check()  # every module that declares switches is imported by now

__all__ = ["HRegNet", "HierFeatureExtraction", "Model_V2", "furthest_point_sample",
           "weighted_furthest_point_sample", "gather_operation", "set_seed", "calc_error_np",
           "knn_points", "knn_gather", "point_utils_cuda", "transformation_loss",
           "calc_rot_rre_err", "calc_tran_rte_err"]
