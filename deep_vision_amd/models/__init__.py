"""Model zoo (reference parity: SURVEY §2.2) and a name -> constructor registry."""
from .classic import VGG16, VGG19, AlexNetV1, AlexNetV2, AlexNetV2TF, LeNet5, LeNet5TF  # noqa: F401
from .inception import InceptionV1, InceptionV3  # noqa: F401
from .mobilenet import MobileNetV1, MobileNetV1TF, ShuffleNetV1  # noqa: F401
from .resnet import ResNet34, ResNet50, ResNet152  # noqa: F401
from .resnet_tf import ResNet50TF, ResNet50V2, ResNet152TF  # noqa: F401
from .yolov3 import YoloV3, Darknet53  # noqa: F401
from .hourglass import StackedHourglassNetwork  # noqa: F401
from .centernet import ObjectsAsPoints  # noqa: F401
from .gan import (CycleGANDiscriminator, CycleGANGenerator, DCGANDiscriminator, DCGANGenerator,  # noqa: F401
                  cyclegan, dcgan)

MODELS = {
    "lenet5": LeNet5,
    "lenet5_tf": LeNet5TF,
    "alexnet1": AlexNetV1,
    "alexnet2": AlexNetV2,
    "alexnet2_tf": AlexNetV2TF,
    "vgg16": VGG16,
    "vgg19": VGG19,
    "inception1": InceptionV1,
    "inception3": InceptionV3,
    "resnet34": ResNet34,
    "resnet50": ResNet50,
    "resnet152": ResNet152,
    "mobilenet1": MobileNetV1,
    "mobilenet1_tf": MobileNetV1TF,
    "shufflenet1": ShuffleNetV1,
    "resnet50_tf": ResNet50TF,
    "resnet152_tf": ResNet152TF,
    "resnet50v2_tf": ResNet50V2,
    "yolov3": YoloV3,
    "darknet53": Darknet53,
    "hourglass104": StackedHourglassNetwork,
    "centernet": ObjectsAsPoints,
    "dcgan_generator": DCGANGenerator,
    "dcgan_discriminator": DCGANDiscriminator,
    "cyclegan_generator": CycleGANGenerator,
    "cyclegan_discriminator": CycleGANDiscriminator,
    "dcgan": dcgan,
    "cyclegan": cyclegan,
}


def register(name):
    def deco(cls):
        MODELS[name] = cls
        return cls

    return deco


def get_model(name: str, **kw):
    try:
        return MODELS[name](**kw)
    except KeyError:
        raise KeyError(f"unknown model {name!r}; available: {sorted(MODELS)}") from None
