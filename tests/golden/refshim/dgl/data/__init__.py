class CiteseerGraphDataset:  # import-only stubs (model/REMixHop.py imports them)
    pass


class CoraGraphDataset:
    pass


class PubmedGraphDataset:
    pass
