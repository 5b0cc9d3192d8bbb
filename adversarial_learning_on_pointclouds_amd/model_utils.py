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


# weight initialisers by init_type (utils/model_utils.py:27-58); biases go to 0
_WEIGHT_INIT = {
    "normal": lambda w, gain: init.normal_(w, 0.0, gain),
    "xavier": lambda w, gain: init.xavier_normal_(w, gain=gain),
    "kaiming": lambda w, gain: init.kaiming_normal_(w, a=0, mode="fan_in"),
    "orthogonal": lambda w, gain: init.orthogonal_(w, gain=gain),
}


def init_weights(net, init_type, init_gain=1.0, verbose=True):
    """Initialise every Conv*/Linear weight of `net` by `init_type` and zero its
    bias; BatchNorm2d weights ~ N(1, init_gain), biases 0 (interface and
    distributions of utils/model_utils.py:27-58).  Leaf modules are visited in
    registration order, the order Module.apply reaches them, so a seeded torch
    RNG gives the reference's weights."""
    if verbose:
        print("initialize network with %s" % init_type)
    if init_type is None:
        return net
    fill = _WEIGHT_INIT.get(init_type)
    for mod in net.modules():
        kind = type(mod).__name__
        if ("Conv" in kind or "Linear" in kind) and hasattr(mod, "weight"):
            if fill is None:
                raise NotImplementedError("initialization method [%s] is not implemented" % init_type)
            fill(mod.weight.data, init_gain)
            if getattr(mod, "bias", None) is not None:
                mod.bias.data.zero_()
        elif "BatchNorm2d" in kind:
            init.normal_(mod.weight.data, 1.0, init_gain)
            mod.bias.data.zero_()
    return net


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
