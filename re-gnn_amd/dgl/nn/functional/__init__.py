from ..pytorch.softmax import edge_softmax  # noqa: F401
