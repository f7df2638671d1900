from .resnet import (BasicBlock, Bottleneck, ResNet, build_model, resnet18, resnet34, resnet50,
                     resnet101, resnet152)

__all__ = ["BasicBlock", "Bottleneck", "ResNet", "build_model", "resnet18", "resnet34",
           "resnet50", "resnet101", "resnet152"]
