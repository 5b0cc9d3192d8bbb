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
from . import _lib  # noqa: E402
from ._lib import use_stream_graph_dispatch  # noqa: E402
from .discriminator import DeepConvDiscNet  # noqa: E402
from .pointnet import PointNetCls, PointNetfeat, STN3d, STNkd, feature_transform_regularizer  # noqa: E402,E501
from .seg import PointNetSeg, SegTrainStep  # noqa: E402
from .step import AdvTrainStep  # noqa: E402

__all__ = ["PointNetCls", "PointNetfeat", "STN3d", "STNkd", "DeepConvDiscNet",
           "feature_transform_regularizer", "AdvTrainStep", "PointNetSeg", "SegTrainStep"]
__version__ = "0.1.0"
