from . import hetero  # noqa: F401


def to_undirected(*a, **k):
    raise NotImplementedError
