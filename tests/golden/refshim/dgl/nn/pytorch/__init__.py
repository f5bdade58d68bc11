from . import softmax, utils, conv  # noqa: F401
