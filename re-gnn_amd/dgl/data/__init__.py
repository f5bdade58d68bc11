"""dgl.data names imported by model/REMixHop.py:15 (citation datasets need a download: absent)."""


class _Offline:
    def __init__(self, *a, **k):
        raise NotImplementedError(f"{type(self).__name__} needs a network download (not available)")


class CiteseerGraphDataset(_Offline):
    pass


class CoraGraphDataset(_Offline):
    pass


class PubmedGraphDataset(_Offline):
    pass
