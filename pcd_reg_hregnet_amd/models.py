"""``HRegNet`` / ``HierFeatureExtraction`` -- drop-in modules for models/HRegNet.

Same constructor arguments (``args.use_fps, use_weights, freeze_detector,
freeze_feats``), the same sub-module tree and therefore the same state-dict
keys as the reference (models/HRegNet/models.py:7-75, layers.py:89-504), so
``ckpt/pretrained/nusc_feats.pth`` and any trained checkpoint load unchanged.
``forward`` returns the reference's dict (models.py:129-148).

The parameters are plain nn.Conv/BatchNorm modules (they are the checkpoint
format); the forward itself runs on the gfx950 HIP library through
:mod:`pcd_reg_hregnet_amd.engine` -- BatchNorm in eval mode.  The training
forward (``HRegNet`` in .train()) runs pcd_reg_hregnet_amd.train_graph: train-mode
BatchNorm and a backward made of HIP kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import engine


def _conv_bn_relu(cin, cout, dims=2, bias=False):
    conv = nn.Conv2d if dims == 2 else nn.Conv1d
    bn = nn.BatchNorm2d if dims == 2 else nn.BatchNorm1d
    return [conv(cin, cout, kernel_size=1, bias=bias), bn(cout), nn.ReLU()]


def _stack(chans, dims=2):
    layers = []
    for a, b in zip(chans[:-1], chans[1:]):
        layers += _conv_bn_relu(a, b, dims)
    return nn.Sequential(*layers)


def _head(C):
    """mlp1/mlp2 = Conv1d(C,C)+BN+ReLU, mlp3 = Conv1d(C,1) (layers.py:124-130)."""
    return (nn.Sequential(*_conv_bn_relu(C, C, 1, bias=True)),
            nn.Sequential(*_conv_bn_relu(C, C, 1, bias=True)),
            nn.Sequential(nn.Conv1d(C, 1, kernel_size=1)))


class _HIPOnly(nn.Module):
    def forward(self, *a, **k):  # pragma: no cover - guidance only
        raise NotImplementedError(
            f"{type(self).__name__} runs fused inside HRegNet/HierFeatureExtraction.forward")


class KeypointDetector(_HIPOnly):
    """Parameter layout of layers.py:89-132."""

    def __init__(self, nsample, k, in_channels, out_channels, fps=True):
        super().__init__()
        self.nsample, self.k, self.fps = nsample, k, fps
        self.convs = _stack([in_channels + 4, *out_channels])
        self.C_o1 = out_channels[-1]
        self.mlp1, self.mlp2, self.mlp3 = _head(self.C_o1)
        self.softplus = nn.Softplus()


class DescExtractor(_HIPOnly):
    """Parameter layout of layers.py:167-198."""

    def __init__(self, in_channels, out_channels, C_detector, desc_dim):
        super().__init__()
        chans = [in_channels + 4, *out_channels]
        self.convs = _stack(chans)
        self.C_o1 = chans[-1]
        self.mlp1 = nn.Sequential(*_conv_bn_relu(2 * self.C_o1 + C_detector, chans[-2]))
        self.mlp2 = nn.Sequential(*_conv_bn_relu(chans[-2], desc_dim))


class CoarseReg(nn.Module):
    """layers.py:229-396: the parameter layout of every (use_sim, use_neighbor) variant --
    convs_1 over 2C + 16 / 14 / 14 / 12 inputs (layers.py:237-244); convs_2 exists in all of them,
    as in the reference -- and, in eval mode, the reference's forward on the HIP library:
    (src_xyz [B,N,3], src_desc [B,C,N], dst_xyz, dst_desc, src_weights [B,N], dst_weights) ->
    (corres_xyz [B,N,3], weights [B,N]).  HRegNet / Model_V2 run the True / True head fused inside
    their own forward; a variant there, or this module alone, runs engine.coarse_reg with the
    variant's absent similarity features as zero columns (engine._pad_coarse_convs1)."""

    def __init__(self, k, in_channels, use_sim=True, use_neighbor=True):
        super().__init__()
        self.k, self.use_sim, self.use_neighbor = k, bool(use_sim), bool(use_neighbor)
        C = in_channels
        extra = 12 + 2 * self.use_sim + 2 * self.use_neighbor
        self.convs_1 = _stack([2 * C + extra, 2 * C, 2 * C, 2 * C])
        self.convs_2 = _stack([C + 4, C, C, C])
        self.mlp1, self.mlp2, self.mlp3 = _head(2 * C)
        self._prep = _Prepared()

    @property
    def variant(self):
        return (self.use_sim, self.use_neighbor)

    def forward(self, src_xyz, src_desc, dst_xyz, dst_desc, src_weights, dst_weights):
        if self.training:
            raise NotImplementedError("CoarseReg alone runs in eval mode (the training step runs "
                                      "inside HRegNet.train(), train_graph.py)")
        B, N, _ = src_xyz.shape
        C = src_desc.shape[1]
        P = self._prep.get(_PrefixedHead(self, "coarse_corres"), src_xyz.device, self.variant)
        xyz3 = torch.cat([src_xyz, dst_xyz]).float().contiguous()
        desc3 = torch.cat([src_desc, dst_desc]).transpose(1, 2).reshape(2 * B * N, C).float().contiguous()
        sig3 = torch.cat([src_weights, dst_weights]).reshape(-1).float().contiguous()
        with torch.no_grad():
            corres, w = engine.coarse_reg(P, B, xyz3, desc3, sig3)
        return corres, w


class FineReg(_HIPOnly):
    """Parameter layout of layers.py:414-431."""

    def __init__(self, k, in_channels):
        super().__init__()
        self.k = k
        C = in_channels
        self.convs_1 = _stack([2 * C + 12, 2 * C, 2 * C, 2 * C])
        self.mlp1, self.mlp2, self.mlp3 = _head(2 * C)


FineReg1 = FineReg  # model_v2/layers.py:368-424 (same layout as FineReg)


class FineReg2(FineReg):
    """Parameter layout of model_v2/layers.py:426-460: FineReg + mlpx (Conv1d 2C->C+BN+ReLU)."""

    def __init__(self, k, in_channels):
        super().__init__(k, in_channels)
        self.mlpx = nn.Sequential(*_conv_bn_relu(2 * in_channels, in_channels, 1, bias=True))


class WeightedSVDHead(nn.Module):
    """layers.py:456-504 on the HIP library: (src, src_corres, weights) -> (R, t)."""

    def forward(self, src, src_corres, weights):
        _, _, R, t = engine.weighted_svd(src.float().contiguous(), src_corres.float().contiguous(),
                                         weights.float().contiguous())
        return R, t


def _weights_key(module: nn.Module, device):
    return (str(device),) + tuple(
        (t.data_ptr(), t._version) for t in module.state_dict(keep_vars=True).values())


class _Prepared:
    """Caches the folded device weights until a parameter or buffer changes."""

    def __init__(self):
        self.key = None
        self.value = None

    def get(self, module, device, coarse_variant=(True, True)):
        key = _weights_key(module, device) + (tuple(coarse_variant),)
        if key != self.key:
            self.value = engine.PreparedWeights(module.state_dict(), device, coarse_variant)
            self.key = key
        return self.value


class HierFeatureExtraction(nn.Module):
    """models/HRegNet/models.py:7-58."""

    def __init__(self, args):
        super().__init__()
        self.use_fps = args.use_fps
        self.use_weights = args.use_weights
        self.detector_1 = KeypointDetector(1024, 64, 0, [32, 32, 64], fps=self.use_fps)
        self.detector_2 = KeypointDetector(512, 32, 64, [64, 64, 128], fps=self.use_fps)
        self.detector_3 = KeypointDetector(256, 16, 128, [128, 128, 256], fps=self.use_fps)
        if args.freeze_detector:
            for p in self.parameters():
                p.requires_grad = False
        self.desc_extractor_1 = DescExtractor(0, [32, 32, 64], 64, 64)
        self.desc_extractor_2 = DescExtractor(64, [64, 64, 128], 128, 128)
        self.desc_extractor_3 = DescExtractor(128, [128, 128, 256], 256, 256)
        self._prep = _Prepared()

    def forward(self, points):
        B = points.shape[0]
        if self.training:
            # (models.py:26-58 in train mode, as train_feats.py trains it: batch-statistics BN,
            # running statistics updated, differentiable in every parameter -- the same
            # train_graph.feature_extraction HRegNet's training step runs for src and dst)
            from . import train_graph
            out = train_graph.feature_extraction_call(self, points.float().contiguous())
            return {k: (v if k.startswith("xyz") else
                        v.view(B, -1) if k.startswith("sigmas") else
                        v.view(B, v.shape[0] // B, -1).transpose(1, 2))
                    for k, v in out.items() if not k.startswith("fps_idx")}
        P = self._prep.get(_Prefixed(self), points.device)
        samples = None if self.use_fps else engine.random_samples(
            1, points.shape[0], engine.level_input_sizes(points.shape[1]), points.device)
        out = engine.feature_extraction(P, points.float().contiguous(), self.use_weights,
                                        samples=samples)
        res = {}
        for i, m in enumerate((1024, 512, 256)):
            res[f"xyz_{i + 1}"] = out[f"xyz_{i + 1}"]
            res[f"sigmas_{i + 1}"] = out[f"sigmas_{i + 1}"].view(B, m)
            res[f"desc_{i + 1}"] = out[f"desc_{i + 1}"].view(B, m, -1).transpose(1, 2).contiguous()
        return res


class _Prefixed(nn.Module):
    """Presents a HierFeatureExtraction's state dict under 'feature_extraction.' with
    dummy (never used) head weights, so PreparedWeights can fold it."""

    def __init__(self, fe):
        super().__init__()
        object.__setattr__(self, "_fe", fe)

    def state_dict(self, *a, keep_vars=False, **k):
        sd = {"feature_extraction." + n: v
              for n, v in self._fe.state_dict(keep_vars=keep_vars).items()}
        sd.update(_dummy_heads())
        return sd


class _PrefixedHead(nn.Module):
    """A registration head's state dict under its HRegNet name (prefix) beside dummy (never
    used) feature-extraction and other head weights, so PreparedWeights can fold it alone."""

    def __init__(self, head, prefix):
        super().__init__()
        object.__setattr__(self, "_h", head)
        object.__setattr__(self, "_prefix", prefix)

    def state_dict(self, *a, keep_vars=False, **k):
        sd = {k_: v for k_, v in _dummy_heads().items() if not k_.startswith(self._prefix + ".")}
        sd.update(_dummy_features())
        sd.update({self._prefix + "." + n: v for n, v in self._h.state_dict(keep_vars=keep_vars).items()
                   if not n.startswith("_")})
        return sd


_DUMMY = None
_DUMMY_FE = None


def _dummy_features():
    global _DUMMY_FE
    if _DUMMY_FE is None:
        class _A:
            use_fps = use_weights = True
            freeze_detector = freeze_feats = False
        with torch.random.fork_rng(devices=[]):
            fe = HierFeatureExtraction(_A())
        _DUMMY_FE = {"feature_extraction." + k: v for k, v in fe.state_dict().items()}
    return _DUMMY_FE


def _dummy_heads():
    global _DUMMY
    if _DUMMY is None:
        with torch.random.fork_rng(devices=[]):
            m = nn.Module()
            m.coarse_corres = CoarseReg(8, 256)
            m.fine_corres_2 = FineReg(8, 128)
            m.fine_corres_1 = FineReg(8, 64)
        _DUMMY = {k: v for k, v in m.state_dict().items()}
    return _DUMMY


class HRegNet(nn.Module):
    """models/HRegNet/models.py:60-148."""

    def __init__(self, args):
        super().__init__()
        self.feature_extraction = HierFeatureExtraction(args)
        if args.freeze_feats:
            for p in self.parameters():
                p.requires_grad = False
        self.coarse_corres = CoarseReg(k=8, in_channels=256, use_sim=True, use_neighbor=True)
        self.fine_corres_2 = FineReg(k=8, in_channels=128)
        self.fine_corres_1 = FineReg(k=8, in_channels=64)
        self.svd_head = WeightedSVDHead()
        self._prep = _Prepared()

    def prepared(self, device):
        return self._prep.get(self, device, self.coarse_corres.variant)

    def forward(self, src_points, dst_points):
        if self.training:
            # batch-statistics BN + backward kernels (train_graph.py, csrc/train_ops.hip)
            from . import train_graph
            return train_graph.hregnet_train_forward(self, src_points, dst_points)
        dev = src_points.device
        P = self.prepared(dev)
        out = engine.hregnet_forward(P, src_points.float().contiguous(),
                                     dst_points.float().contiguous(),
                                     self.feature_extraction.use_weights,
                                     use_fps=self.feature_extraction.use_fps)
        engine.check_device_status()  # syncs only when a multi-workgroup FPS ran (N > 16384)
        out.pop("_fps_idx", None)
        for part in ("src_feats", "dst_feats"):
            out[part] = {k: v.contiguous() for k, v in out[part].items()}
        return out


class Model_V2(nn.Module):
    """models/model_v2/models.py:60-183 (inference): HRegNet with FineReg2 (mlpx
    features + batch-shuffled "prime" copies for the MI loss)."""

    def __init__(self, args):
        super().__init__()
        self.feature_extraction = HierFeatureExtraction(args)
        if args.freeze_feats:
            for p in self.parameters():
                p.requires_grad = False
        self.coarse_corres = CoarseReg(k=8, in_channels=256, use_sim=True, use_neighbor=True)
        self.fine_corres_2 = FineReg2(k=8, in_channels=128)
        self.fine_corres_1 = FineReg1(k=8, in_channels=64)
        self.svd_head = WeightedSVDHead()
        self._prep = _Prepared()

    def prepared(self, device):
        return self._prep.get(self, device, self.coarse_corres.variant)

    def forward(self, src_points, dst_points):
        if self.training:
            # batch-statistics BN + backward kernels (train_graph.py, csrc/train_ops.hip)
            from . import train_graph
            return train_graph.hregnet_train_forward(self, src_points, dst_points, v2=True)
        P = self.prepared(src_points.device)
        out = engine.model_v2_forward(P, src_points.float().contiguous(),
                                      dst_points.float().contiguous(),
                                      self.feature_extraction.use_weights,
                                      use_fps=self.feature_extraction.use_fps)
        engine.check_device_status()  # syncs only when a multi-workgroup FPS ran (N > 16384)
        out.pop("_fps_idx", None)
        for key in ("src_feats_desc_2", "src_dst_feats_2", "src_dst_feats_2_prime"):
            out[key] = out[key].contiguous()
        for part in ("src_feats", "dst_feats"):
            out[part] = {k: v.contiguous() for k, v in out[part].items()}
        return out
