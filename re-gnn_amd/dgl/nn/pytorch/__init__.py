from . import softmax, utils, conv  # noqa: F401
from .softmax import edge_softmax  # noqa: F401
