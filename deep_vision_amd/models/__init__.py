"""Model zoo (reference parity: SURVEY §2.2) and a name -> constructor registry."""
from .resnet import ResNet34, ResNet50, ResNet152  # noqa: F401

MODELS = {
    "resnet34": ResNet34,
    "resnet50": ResNet50,
    "resnet152": ResNet152,
}


def get_model(name: str, **kw):
    try:
        return MODELS[name](**kw)
    except KeyError:
        raise KeyError(f"unknown model {name!r}; available: {sorted(MODELS)}") from None
