"""Model factory and init (utils/model_utils.py:12-140), same signatures."""
from __future__ import annotations

import sys

import torch
from torch.nn import init

from .discriminator import DeepConvDiscNet
from .pointnet import PointNetCls


def init_net(net, device, init_type, init_gain=1.0):
    """utils/model_utils.py:12-25: move to device, then init_weights."""
    net.to(device)
    if init_type is None:
        return net
    init_weights(net, init_type, init_gain=init_gain)
    return net


def init_weights(net, init_type, init_gain=1.0, verbose=True):
    """utils/model_utils.py:27-58: Conv/Linear weights by init_type, biases 0."""
    def init_func(m):
        classname = m.__class__.__name__
        if hasattr(m, "weight") and (classname.find("Conv") != -1 or classname.find("Linear") != -1):
            if init_type == "normal":
                init.normal_(m.weight.data, 0.0, init_gain)
            elif init_type == "xavier":
                init.xavier_normal_(m.weight.data, gain=init_gain)
            elif init_type == "kaiming":
                init.kaiming_normal_(m.weight.data, a=0, mode="fan_in")
            elif init_type == "orthogonal":
                init.orthogonal_(m.weight.data, gain=init_gain)
            else:
                raise NotImplementedError("initialization method [%s] is not implemented" % init_type)
            if hasattr(m, "bias") and m.bias is not None:
                init.constant_(m.bias.data, 0.0)
        elif classname.find("BatchNorm2d") != -1:
            init.normal_(m.weight.data, 1.0, init_gain)
            init.constant_(m.bias.data, 0.0)

    if verbose:
        print("initialize network with %s" % init_type)
    if init_type is None:
        return net
    net.apply(init_func)


def load_models(mode, device, args):
    """utils/model_utils.py:60-140 for the hot path's modes 'cls' and 'disc' and
    the segmentation row's 'seg'.
    The segmentation / stacked discriminators are outside this build's scope."""
    if mode == "cls":
        model = PointNetCls(k=40, feature_transform=False).to(device)
        try:
            if getattr(args, "checkpoint", None):
                print("===============================")
                print("Loading pretrained cls model ...")
                print("===============================")
                model.load_state_dict(torch.load(args.checkpoint, map_location=device,
                                                 weights_only=True))
        except Exception as e:  # reference: print and exit(0) (:77-79)
            print(e)
            sys.exit(0)
    elif mode == "disc":
        model = DeepConvDiscNet(input_dim=args.disc_indim, output_dim=1)
        model = init_net(model, device, init_type=args.init_disc)
    elif mode == "seg":  # :80-90, PointNetSeg
        from .seg import PointNetSeg
        model = PointNetSeg(NUM_SEG_CLASSES=50)
        model = init_net(model, device, init_type=args.init_disc)
        if getattr(args, "checkpoint", None):
            print("Loading pretrained cls model ...")
            model.load_state_dict(torch.load(args.checkpoint, map_location=device,
                                             weights_only=True))
    elif mode in ("seg_regu", "disc_seg", "disc_dual", "disc_stack"):
        raise NotImplementedError(f"mode {mode!r} is outside the adversarial cls hot path")
    else:
        raise ValueError("Invalid mode {}!".format(mode))
    return model
