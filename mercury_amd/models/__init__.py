"""Model zoo (reference `pytorch_model.py` + BASELINE additions)."""
from .resnet import (BasicBlock, Bottleneck, ResNet, ResNet18, ResNet34, ResNet50,
                     ResNet101, ResNet152, ResNet50_ImageNet)
from .vgg import VGG, cfg as vgg_cfg
from .lstm import Attention, MyLSTM
from .mobilenetv2 import MobileNetV2, InvertedResidual

_FACTORIES = {
    'resnet18': ResNet18, 'resnet34': ResNet34, 'resnet50': ResNet50,
    'resnet101': ResNet101, 'resnet152': ResNet152,
    'resnet50_imagenet': ResNet50_ImageNet, 'mobilenetv2': MobileNetV2,
}


def build_model(name, num_classes=10):
    name = name.lower()
    if name.startswith('vgg'):
        return VGG(name.upper(), num_classes)
    if name in ('resnet', 'resnet-18'):
        name = 'resnet18'
    return _FACTORIES[name](num_classes)


__all__ = ['BasicBlock', 'Bottleneck', 'ResNet', 'ResNet18', 'ResNet34', 'ResNet50',
           'ResNet101', 'ResNet152', 'ResNet50_ImageNet', 'VGG', 'vgg_cfg', 'Attention',
           'MyLSTM', 'MobileNetV2', 'InvertedResidual', 'build_model']
