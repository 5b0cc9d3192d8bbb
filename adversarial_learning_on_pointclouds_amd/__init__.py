"""MI355X-native PointNet adversarial-training hot path (gfx950 HIP kernels).

Drop-in counterparts of the reference's models and training loop
(YiruS/Adversarial_Learning_on_PointClouds): PointNetCls / PointNetfeat
(models/pointnet.py), DeepConvDiscNet (models/discriminator.py), load_models
(utils/model_utils.py), make_D_label (utils/utils.py), ImagePool
(utils/image_pool.py), run_training / run_testing (utils/trainer.py), plus the
fused native step AdvTrainStep; PointNetSeg (models/pointnet.py:261-317) with
its native training step SegTrainStep; run_training_semi; the HDF5 datasets of
dataset/modelNetData.py and dataset/shapeNetData.py without h5py, with a
device-resident batch loader (dataset.DeviceCloudLoader).  All compute runs in
libpcadv.so (C ABI in include/pcadv.h); there is no CPU fallback.
"""
import os as _os

# HIP graphs of the step replay faster when the runtime dispatches their nodes
# through the stream path instead of pre-recorded AQL packets (measured on
# MI355X, ROCm 7: adv step -2.5 %, cls -3.5 %, seg unchanged).
# Read once at HIP runtime initialisation, so it only takes effect when this
# package is imported before the first GPU call; PCADV_GRAPH_PACKET_CAPTURE=1
# (or setting DEBUG_CLR_GRAPH_PACKET_CAPTURE yourself) keeps the runtime default.
if _os.environ.get("PCADV_GRAPH_PACKET_CAPTURE", "0") != "1":
    _os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

from . import _lib  # noqa: E402
from .discriminator import DeepConvDiscNet  # noqa: E402
from .pointnet import PointNetCls, PointNetfeat, STN3d, STNkd, feature_transform_regularizer  # noqa: E402,E501
from .seg import PointNetSeg, SegTrainStep  # noqa: E402
from .step import AdvTrainStep  # noqa: E402

__all__ = ["PointNetCls", "PointNetfeat", "STN3d", "STNkd", "DeepConvDiscNet",
           "feature_transform_regularizer", "AdvTrainStep", "PointNetSeg", "SegTrainStep"]
__version__ = "0.1.0"
