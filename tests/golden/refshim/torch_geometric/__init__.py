from . import nn, utils, loader  # noqa: F401
